package org.redisson;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.lang.invoke.MethodHandle;
import org.redisson.api.RBloomFilter;
import org.redisson.api.RHyperLogLog;
import org.redisson.client.codec.Codec;
import static java.lang.foreign.ValueLayout.*;

/**
 * RedissonClient.getBloomFilter / getHyperLogLog (M/Redisson.java:235-241,658-664) on a node's GPUs: the
 * objects the wrapped client would build, with their hot path on the GPU that owns the name's Redis Cluster
 * slot (calcSlot(name) * nGpus / 16384, include/rbx.h rbx_node_gpu_of).  Codecs and the executor (for the
 * RObject plumbing the shim does not replace) come from the wrapped client.
 */
public final class GpuRedisson implements AutoCloseable {
    private final MemorySegment node;                           // rbx_node* over this node's GPUs
    private final Redisson redisson;                            // codecs and executor of the wrapped client

    public GpuRedisson(Redisson redisson, int nGpus) {
        this.redisson = redisson;
        try (Arena a = Arena.ofConfined()) {
            MemorySegment out = a.allocate(ADDRESS);
            MethodHandle init = Rbx.h("rbx_node_init", JAVA_INT, JAVA_INT, ADDRESS, ADDRESS);
            Rbx.check((int) init.invokeExact(nGpus, MemorySegment.NULL, out));
            node = out.get(ADDRESS, 0);
        } catch (Throwable t) { throw Rbx.rethrow(t); }
    }

    /** The context of the GPU owning `name`'s slot (rbx_node_gpu_of + rbx_node_ctx). */
    MemorySegment ctxOf(String name) {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment g = a.allocate(JAVA_INT), c = a.allocate(ADDRESS);
            Rbx.check((int) Rbx.h("rbx_node_gpu_of", JAVA_INT, ADDRESS, Rbx.NAME, ADDRESS)
                    .invokeExact(node, Rbx.name(a, name), g));
            Rbx.check((int) Rbx.h("rbx_node_ctx", JAVA_INT, ADDRESS, JAVA_INT, ADDRESS)
                    .invokeExact(node, g.get(JAVA_INT, 0), c));
            return c.get(ADDRESS, 0);
        } catch (Throwable t) { throw Rbx.rethrow(t); }
    }

    public <V> RBloomFilter<V> getBloomFilter(String name) {                   // M/Redisson.java:658-661
        return getBloomFilter(name, redisson.getConfig().getCodec());
    }

    public <V> RBloomFilter<V> getBloomFilter(String name, Codec codec) {      // M/Redisson.java:663-666
        return new GpuBloomFilter<>(codec, redisson.getCommandExecutor(), name, ctxOf(name));
    }

    public <V> RHyperLogLog<V> getHyperLogLog(String name) {                   // M/Redisson.java:235-238
        return getHyperLogLog(name, redisson.getConfig().getCodec());
    }

    public <V> RHyperLogLog<V> getHyperLogLog(String name, Codec codec) {      // M/Redisson.java:240-243
        return new GpuHyperLogLog<>(codec, redisson.getCommandExecutor(), name, ctxOf(name));
    }

    @Override public void close() {                                           // rbx_node_shutdown
        try {
            MethodHandle down = Rbx.h("rbx_node_shutdown", JAVA_INT, ADDRESS);
            Rbx.check((int) down.invokeExact(node));
        } catch (Throwable t) { throw Rbx.rethrow(t); }
    }
}
