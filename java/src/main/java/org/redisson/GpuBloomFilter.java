package org.redisson;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.lang.invoke.MethodHandle;
import java.util.ArrayList;
import java.util.Collection;
import java.util.List;
import org.redisson.api.RBloomFilter;
import org.redisson.client.codec.Codec;
import org.redisson.command.CommandAsyncExecutor;
import static java.lang.foreign.ValueLayout.*;

/**
 * Drop-in for RedissonBloomFilter (M/RedissonBloomFilter.java), one instance per name like the reference:
 * the hashing, the k bit indexes and the SETBIT / GETBIT batch run on the GPU behind librbx.so
 * (include/rbx.h rbx_bloom_*_n); the codec stays here (RedissonObject.encode, M/RedissonObject.java:319-321).
 */
public class GpuBloomFilter<T> extends GpuExpirable implements RBloomFilter<T> {
    private final String configName;          // suffixName(name, "config") (:75)
    private volatile long size;               // cached like :61-62
    private volatile int hashIterations;

    public GpuBloomFilter(Codec codec, CommandAsyncExecutor ex, String name, MemorySegment ctx) {
        super(codec, ex, name, ctx);
        this.configName = suffixName(getRawName(), "config");
    }

    @Override protected String[] keyNames() { return new String[] {getRawName(), configName}; }

    @Override public boolean tryInit(long expectedInsertions, double falseProbability) {   // :262-300
        try (Arena a = Arena.ofConfined()) {
            MemorySegment created = a.allocate(JAVA_INT);
            Rbx.check((int) Rbx.TRY_INIT.invokeExact(ctx, Rbx.name(a, getRawName()), expectedInsertions,
                    falseProbability, created));
            readConfig();
            return created.get(JAVA_INT, 0) != 0;
        } catch (Throwable t) { throw Rbx.rethrow(t); }
    }

    @Override public long add(Collection<T> objects) { return batch(Rbx.ADD, objects); }           // :104-137
    @Override public long contains(Collection<T> objects) { return batch(Rbx.CONTAINS, objects); }  // :153-186
    @Override public boolean add(T object) { return add(List.of(object)) > 0; }                     // :99-102
    @Override public boolean contains(T object) { return contains(List.of(object)) > 0; }           // :198-201

    private long batch(MethodHandle op, Collection<T> objects) {
        if (size == 0) readConfig();                                          // :106-108
        try (Arena a = Arena.ofConfined()) {
            List<byte[]> enc = new ArrayList<>(objects.size());
            for (T o : objects) {                                             // RedissonObject.encode (:319-321)
                io.netty.buffer.ByteBuf b = encode(o);
                try { byte[] x = new byte[b.readableBytes()]; b.getBytes(b.readerIndex(), x); enc.add(x); }
                finally { b.release(); }
            }
            MemorySegment count = a.allocate(JAVA_LONG);
            Rbx.check((int) op.invokeExact(ctx, Rbx.name(a, getRawName()), size, hashIterations,
                    Rbx.keys(a, enc), MemorySegment.NULL, count));
            return count.get(JAVA_LONG, 0);
        } catch (Throwable t) { throw Rbx.rethrow(t); }
    }

    @Override public long count() {                                             // :215-227
        try (Arena a = Arena.ofConfined()) {
            MemorySegment out = a.allocate(JAVA_LONG);
            Rbx.check((int) Rbx.COUNT.invokeExact(ctx, Rbx.name(a, getRawName()), out));
            readConfig();
            return out.get(JAVA_LONG, 0);
        } catch (Throwable t) { throw Rbx.rethrow(t); }
    }

    /** readConfig() :240-255: HGETALL {name}:config -> the cached size / hashIterations. */
    private MemorySegment readConfig(Arena a) throws Throwable {
        MemorySegment cfg = a.allocate(Rbx.CONFIG);
        Rbx.check((int) Rbx.READ_CONFIG.invokeExact(ctx, Rbx.name(a, getRawName()), cfg));  // ISE when absent (:251)
        size = cfg.get(JAVA_LONG, Rbx.CONFIG_SIZE_BITS);
        hashIterations = cfg.get(JAVA_INT, Rbx.CONFIG_K);
        return cfg;
    }

    private void readConfig() {
        try (Arena a = Arena.ofConfined()) { readConfig(a); } catch (Throwable t) { throw Rbx.rethrow(t); }
    }

    @Override public long getExpectedInsertions() {                            // :318-322 (HGET expectedInsertions)
        try (Arena a = Arena.ofConfined()) { return readConfig(a).get(JAVA_LONG, Rbx.CONFIG_EXPECTED); }
        catch (Throwable t) { throw Rbx.rethrow(t); }
    }

    @Override public double getFalseProbability() {                            // Double.valueOf(the plain string)
        try (Arena a = Arena.ofConfined()) { return Double.parseDouble(readConfig(a).getString(Rbx.CONFIG_FPP_STR)); }
        catch (Throwable t) { throw Rbx.rethrow(t); }
    }

    @Override public long getSize() { readConfig(); return size; }
    @Override public int getHashIterations() { readConfig(); return hashIterations; }
}
