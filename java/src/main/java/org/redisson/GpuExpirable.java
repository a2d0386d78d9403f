package org.redisson;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.lang.invoke.MethodHandle;
import java.util.concurrent.TimeUnit;
import org.redisson.api.RFuture;
import org.redisson.command.CommandAsyncExecutor;
import org.redisson.client.codec.Codec;
import org.redisson.misc.CompletableFutureWrapper;
import static java.lang.foreign.ValueLayout.*;

/**
 * RObject / RExpirable over the engine's keyspace for a GPU-resident object: every method acts on all of
 * the object's Redis keys at once, as the reference's overrides do (M/RedissonBloomFilter.java:230-385 for
 * {name} and {name}:config; M/RedissonExpirable.java:53-251 for a single key).  Package org.redisson:
 * RedissonExpirable and its constructor are package-private (M/RedissonExpirable.java:37-45).
 */
abstract class GpuExpirable extends RedissonExpirable {
    protected final MemorySegment ctx;  // rbx_ctx* of the GPU owning this name's slot

    GpuExpirable(Codec codec, CommandAsyncExecutor ex, String name, MemorySegment ctx) {
        super(codec, ex, name);
        this.ctx = ctx;
    }

    /** The object's Redis keys, its own name first. */
    protected abstract String[] keyNames();

    @Override public RFuture<Boolean> deleteAsync() {                           // DEL k1..kn
        try (Arena a = Arena.ofConfined()) {
            String[] k = keyNames();
            MemorySegment n = a.allocate(JAVA_INT);
            Rbx.check((int) Rbx.DEL.invokeExact(ctx, Rbx.names(a, k), k.length, n));
            return new CompletableFutureWrapper<>(n.get(JAVA_INT, 0) > 0);
        } catch (Throwable t) { return new CompletableFutureWrapper<>(Rbx.rethrow(t)); }
    }

    @Override public RFuture<Boolean> isExistsAsync() {                         // EXISTS k1..kn
        try (Arena a = Arena.ofConfined()) {
            String[] k = keyNames();
            MemorySegment n = a.allocate(JAVA_INT);
            Rbx.check((int) Rbx.EXISTS.invokeExact(ctx, Rbx.names(a, k), k.length, n));
            return new CompletableFutureWrapper<>(n.get(JAVA_INT, 0) > 0);
        } catch (Throwable t) { return new CompletableFutureWrapper<>(Rbx.rethrow(t)); }
    }

    @Override public RFuture<Long> sizeInMemoryAsync() {                        // M/RedissonBloomFilter.java:234-238
        try (Arena a = Arena.ofConfined()) {
            String[] k = keyNames();
            MemorySegment out = a.allocate(JAVA_LONG);
            Rbx.check((int) Rbx.SIZE_IN_MEMORY.invokeExact(ctx, Rbx.names(a, k), k.length, out));
            return new CompletableFutureWrapper<>(out.get(JAVA_LONG, 0));
        } catch (Throwable t) { return new CompletableFutureWrapper<>(Rbx.rethrow(t)); }
    }

    @Override public RFuture<Void> renameAsync(String newName) {               // M/RedissonBloomFilter.java:347-362
        try (Arena a = Arena.ofConfined()) {
            Rbx.check((int) Rbx.RENAME.invokeExact(ctx, a.allocateFrom(getRawName()), a.allocateFrom(newName)));
            setName(newName);
            return new CompletableFutureWrapper<>((Void) null);
        } catch (Throwable t) { return new CompletableFutureWrapper<>(Rbx.rethrow(t)); }
    }

    @Override public RFuture<Boolean> renamenxAsync(String newName) {          // M/RedissonBloomFilter.java:364-385
        try (Arena a = Arena.ofConfined()) {
            MemorySegment r = a.allocate(JAVA_INT);
            Rbx.check((int) Rbx.RENAMENX.invokeExact(ctx, a.allocateFrom(getRawName()), a.allocateFrom(newName), r));
            boolean ok = r.get(JAVA_INT, 0) != 0;
            if (ok) setName(newName);
            return new CompletableFutureWrapper<>(ok);
        } catch (Throwable t) { return new CompletableFutureWrapper<>(Rbx.rethrow(t)); }
    }

    private static int cond(String param) {                                   // "" NX XX GT LT
        return switch (param) { case "NX" -> 1; case "XX" -> 2; case "GT" -> 3; case "LT" -> 4; default -> 0; };
    }

    @Override protected RFuture<Boolean> expireAsync(long ttl, TimeUnit unit, String param, String... keys) {
        return pexpire(unit.toMillis(ttl), 0, param);                           // M/RedissonExpirable.java:207-222
    }

    @Override protected RFuture<Boolean> expireAtAsync(long timestamp, String param, String... keys) {
        return pexpire(timestamp, 1, param);                                    // :224-239
    }

    private RFuture<Boolean> pexpire(long when, int absolute, String param) {
        try (Arena a = Arena.ofConfined()) {
            String[] k = keyNames();
            MemorySegment r = a.allocate(JAVA_INT);
            Rbx.check((int) Rbx.PEXPIRE.invokeExact(ctx, Rbx.names(a, k), k.length, when, absolute, cond(param), r));
            return new CompletableFutureWrapper<>(r.get(JAVA_INT, 0) == 1);
        } catch (Throwable t) { return new CompletableFutureWrapper<>(Rbx.rethrow(t)); }
    }

    @Override public RFuture<Boolean> clearExpireAsync() {                     // PERSIST k1..kn (:241-251)
        try (Arena a = Arena.ofConfined()) {
            String[] k = keyNames();
            MemorySegment names = a.allocate(ADDRESS, k.length);
            for (int i = 0; i < k.length; i++) names.setAtIndex(ADDRESS, i, a.allocateFrom(k[i]));
            MemorySegment r = a.allocate(JAVA_INT);
            Rbx.check((int) Rbx.PERSIST.invokeExact(ctx, names, k.length, r));
            return new CompletableFutureWrapper<>(r.get(JAVA_INT, 0) == 1);
        } catch (Throwable t) { return new CompletableFutureWrapper<>(Rbx.rethrow(t)); }
    }

    @Override public RFuture<Long> remainTimeToLiveAsync() { return ttl(Rbx.PTTL); }       // PTTL name (:193-195)
    @Override public RFuture<Long> getExpireTimeAsync() { return ttl(Rbx.PEXPIRETIME); }   // PEXPIRETIME name (:203-205)

    private RFuture<Long> ttl(MethodHandle op) {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment out = a.allocate(JAVA_LONG);
            Rbx.check((int) op.invokeExact(ctx, a.allocateFrom(getRawName()), out));
            return new CompletableFutureWrapper<>(out.get(JAVA_LONG, 0));
        } catch (Throwable t) { return new CompletableFutureWrapper<>(Rbx.rethrow(t)); }
    }
}
