package org.redisson;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.util.ArrayList;
import java.util.Collection;
import java.util.List;
import java.util.concurrent.CompletableFuture;
import org.redisson.api.RFuture;
import org.redisson.api.RHyperLogLog;
import org.redisson.client.codec.Codec;
import org.redisson.command.CommandAsyncExecutor;
import org.redisson.misc.CompletableFutureWrapper;
import static java.lang.foreign.ValueLayout.*;

/** Drop-in for RedissonHyperLogLog (M/RedissonHyperLogLog.java:71-102), async forms included. */
public class GpuHyperLogLog<V> extends GpuExpirable implements RHyperLogLog<V> {
    public GpuHyperLogLog(Codec codec, CommandAsyncExecutor ex, String name, MemorySegment ctx) {
        super(codec, ex, name, ctx);
    }

    @Override protected String[] keyNames() { return new String[] {getRawName()}; }

    private List<byte[]> encodeAll(Collection<V> objects) {
        List<byte[]> enc = new ArrayList<>(objects.size());
        for (V o : objects) {
            io.netty.buffer.ByteBuf b = encode(o);
            try { byte[] x = new byte[b.readableBytes()]; b.getBytes(b.readerIndex(), x); enc.add(x); }
            finally { b.release(); }
        }
        return enc;
    }

    // ---- RHyperLogLogAsync: queued on the context's executor; the upcall completes the future --------
    @Override public RFuture<Boolean> addAsync(V obj) { return addAllAsync(List.of(obj)); }

    @Override public RFuture<Boolean> addAllAsync(Collection<V> objects) {     // PFADD name e1..en
        Arena a = Arena.ofShared();                                             // lives until the upcall
        try {
            MemorySegment keys = Rbx.keys(a, encodeAll(objects));
            MemorySegment names = a.allocate(ADDRESS, 1);
            names.setAtIndex(ADDRESS, 0, a.allocateFrom(getRawName()));
            MemorySegment seg = a.allocate(JAVA_LONG, 2);
            seg.setAtIndex(JAVA_LONG, 1, keys.get(JAVA_LONG, Rbx.KEYS_N));
            MemorySegment changed = a.allocate(JAVA_BYTE);
            long[] ticket = new long[1];
            CompletableFuture<Boolean> cf = Rbx.pending(a, () -> changed.get(JAVA_BYTE, 0) != 0, ticket);
            MemorySegment fut = a.allocate(ADDRESS);
            Rbx.check((int) Rbx.HLL_ADD_ASYNC.invokeExact(ctx, names, 1, seg, keys, changed, Rbx.CALLBACK,
                    MemorySegment.ofAddress(ticket[0]), fut));
            int freed = (int) Rbx.FUTURE_FREE.invokeExact(fut.get(ADDRESS, 0));                   // completion arrives by the upcall
            return new CompletableFutureWrapper<>(cf);
        } catch (Throwable t) { a.close(); return new CompletableFutureWrapper<>(Rbx.rethrow(t)); }
    }

    @Override public RFuture<Long> countAsync() { return countWithAsync(); }

    @Override public RFuture<Long> countWithAsync(String... otherLogNames) {  // PFCOUNT name o1..on
        Arena a = Arena.ofShared();
        try {
            MemorySegment names = a.allocate(ADDRESS, 1 + otherLogNames.length);
            names.setAtIndex(ADDRESS, 0, a.allocateFrom(getRawName()));
            for (int i = 0; i < otherLogNames.length; i++) names.setAtIndex(ADDRESS, i + 1, a.allocateFrom(otherLogNames[i]));
            MemorySegment out = a.allocate(JAVA_LONG);
            long[] ticket = new long[1];
            CompletableFuture<Long> cf = Rbx.pending(a, () -> out.get(JAVA_LONG, 0), ticket);
            MemorySegment fut = a.allocate(ADDRESS);
            Rbx.check((int) Rbx.HLL_COUNT_ASYNC.invokeExact(ctx, names, 1 + otherLogNames.length, out, Rbx.CALLBACK,
                    MemorySegment.ofAddress(ticket[0]), fut));
            int freed = (int) Rbx.FUTURE_FREE.invokeExact(fut.get(ADDRESS, 0));
            return new CompletableFutureWrapper<>(cf);
        } catch (Throwable t) { a.close(); return new CompletableFutureWrapper<>(Rbx.rethrow(t)); }
    }

    @Override public RFuture<Void> mergeWithAsync(String... otherLogNames) {   // PFMERGE name o1..on
        Arena a = Arena.ofShared();
        try {
            MemorySegment srcs = a.allocate(ADDRESS, Math.max(1, otherLogNames.length));
            for (int i = 0; i < otherLogNames.length; i++) srcs.setAtIndex(ADDRESS, i, a.allocateFrom(otherLogNames[i]));
            long[] ticket = new long[1];
            CompletableFuture<Void> cf = Rbx.pending(a, () -> null, ticket);
            MemorySegment fut = a.allocate(ADDRESS);
            Rbx.check((int) Rbx.HLL_MERGE_ASYNC.invokeExact(ctx, a.allocateFrom(getRawName()), srcs, otherLogNames.length,
                    Rbx.CALLBACK, MemorySegment.ofAddress(ticket[0]), fut));
            int freed = (int) Rbx.FUTURE_FREE.invokeExact(fut.get(ADDRESS, 0));
            return new CompletableFutureWrapper<>(cf);
        } catch (Throwable t) { a.close(); return new CompletableFutureWrapper<>(Rbx.rethrow(t)); }
    }

    // ---- RHyperLogLog: the synchronous forms block on the async ones, as RedissonHyperLogLog does -----
    @Override public boolean add(V obj) { return get(addAsync(obj)); }
    @Override public boolean addAll(Collection<V> objects) { return get(addAllAsync(objects)); }
    @Override public long count() { return get(countAsync()); }
    @Override public long countWith(String... otherLogNames) { return get(countWithAsync(otherLogNames)); }
    @Override public void mergeWith(String... otherLogNames) { get(mergeWithAsync(otherLogNames)); }
}
