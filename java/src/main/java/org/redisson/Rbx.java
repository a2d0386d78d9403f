package org.redisson;

import java.lang.foreign.*;
import java.lang.invoke.MethodHandle;
import java.lang.invoke.MethodHandles;
import java.lang.invoke.MethodType;
import java.util.List;
import java.util.Map;
import java.util.concurrent.CompletableFuture;
import java.util.concurrent.ConcurrentHashMap;
import java.util.concurrent.atomic.AtomicLong;
import org.redisson.client.RedisException;
import static java.lang.foreign.ValueLayout.*;

/** Layouts, downcall handles and the error mapping of include/rbx.h. */
final class Rbx {
    static final Linker L = Linker.nativeLinker();
    static final SymbolLookup LIB = SymbolLookup.libraryLookup(System.getProperty("rbx.lib", "librbx.so"), Arena.global());

    // Byte offsets of the structs of include/rbx.h that the shim reads and writes.  tests/c/ffm_replay.c is
    // compiled against these constants (tests/c/java_layout.py extracts them) and checks each one against
    // offsetof / sizeof of the C declarations; the static block below checks them against the layouts.
    static final long KEYS_SIZE = 32, KEYS_BYTES = 0, KEYS_OFFSETS = 8, KEYS_STRIDE = 16, KEYS_N = 24;
    static final long CONFIG_SIZE = 96, CONFIG_SIZE_BITS = 0, CONFIG_K = 8, CONFIG_EXPECTED = 16, CONFIG_FPP = 24,
            CONFIG_FPP_STR = 32;
    static final long NAME_SIZE = 16, NAME_BYTES = 0, NAME_LEN = 8;

    // struct rbx_keys { const uint8_t *bytes; const uint64_t *offsets; uint64_t stride; uint64_t n; }  32 bytes
    static final StructLayout KEYS = MemoryLayout.structLayout(ADDRESS.withName("bytes"), ADDRESS.withName("offsets"),
            JAVA_LONG.withName("stride"), JAVA_LONG.withName("n"));
    // struct rbx_bloom_config { int64 size; uint32 k; (pad 4); int64 expected; double fpp; char fpp_str[64]; }  96 bytes
    static final StructLayout CONFIG = MemoryLayout.structLayout(JAVA_LONG.withName("size"),
            JAVA_INT.withName("hash_iterations"), MemoryLayout.paddingLayout(4), JAVA_LONG.withName("expected_insertions"),
            JAVA_DOUBLE.withName("false_probability"), MemoryLayout.sequenceLayout(64, JAVA_BYTE).withName("false_probability_str"));
    // struct rbx_name { const uint8_t *bytes; uint64_t len; }  16 bytes, passed BY VALUE
    static final StructLayout NAME = MemoryLayout.structLayout(ADDRESS.withName("bytes"), JAVA_LONG.withName("len"));

    static {
        if (KEYS.byteSize() != KEYS_SIZE || off(KEYS, "offsets") != KEYS_OFFSETS || off(KEYS, "stride") != KEYS_STRIDE
                || off(KEYS, "n") != KEYS_N || CONFIG.byteSize() != CONFIG_SIZE || off(CONFIG, "hash_iterations") != CONFIG_K
                || off(CONFIG, "expected_insertions") != CONFIG_EXPECTED || off(CONFIG, "false_probability") != CONFIG_FPP
                || off(CONFIG, "false_probability_str") != CONFIG_FPP_STR || NAME.byteSize() != NAME_SIZE
                || off(NAME, "len") != NAME_LEN)
            throw new ExceptionInInitializerError("rbx struct layouts disagree with their offset constants");
    }

    private static long off(StructLayout l, String field) {
        return l.byteOffset(MemoryLayout.PathElement.groupElement(field));
    }

    static MethodHandle h(String name, MemoryLayout res, MemoryLayout... args) {
        return L.downcallHandle(LIB.find(name).orElseThrow(), FunctionDescriptor.of(res, args));
    }

    static final MethodHandle INIT = h("rbx_init", JAVA_INT, JAVA_INT, ADDRESS);
    static final MethodHandle SHUTDOWN = h("rbx_shutdown", JAVA_INT, ADDRESS);
    static final MethodHandle LAST_ERROR = h("rbx_last_error", ADDRESS);
    // Bloom (binary-safe *_n forms: Redis keys may hold any byte)
    static final MethodHandle TRY_INIT = h("rbx_bloom_try_init_n", JAVA_INT, ADDRESS, NAME, JAVA_LONG, JAVA_DOUBLE, ADDRESS);
    static final MethodHandle READ_CONFIG = h("rbx_bloom_read_config_n", JAVA_INT, ADDRESS, NAME, ADDRESS);
    static final MethodHandle ADD = h("rbx_bloom_add_n", JAVA_INT, ADDRESS, NAME, JAVA_LONG, JAVA_INT, ADDRESS, ADDRESS, ADDRESS);
    static final MethodHandle CONTAINS = h("rbx_bloom_contains_n", JAVA_INT, ADDRESS, NAME, JAVA_LONG, JAVA_INT, ADDRESS, ADDRESS, ADDRESS);
    static final MethodHandle COUNT = h("rbx_bloom_count_n", JAVA_INT, ADDRESS, NAME, ADDRESS);
    static final MethodHandle SIZE_IN_MEMORY = h("rbx_memory_usage_n", JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS);
    // keys of any type
    static final MethodHandle DEL = h("rbx_del_n", JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS);
    static final MethodHandle EXISTS = h("rbx_exists_n", JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS);
    static final MethodHandle RENAME = h("rbx_bloom_rename", JAVA_INT, ADDRESS, ADDRESS, ADDRESS);
    static final MethodHandle RENAMENX = h("rbx_bloom_renamenx", JAVA_INT, ADDRESS, ADDRESS, ADDRESS, ADDRESS);
    static final MethodHandle PEXPIRE = h("rbx_pexpire_n", JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, JAVA_LONG, JAVA_INT, JAVA_INT, ADDRESS);
    static final MethodHandle PERSIST = h("rbx_persist", JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS);
    static final MethodHandle PTTL = h("rbx_pttl", JAVA_INT, ADDRESS, ADDRESS, ADDRESS);
    static final MethodHandle PEXPIRETIME = h("rbx_pexpiretime", JAVA_INT, ADDRESS, ADDRESS, ADDRESS);
    // HyperLogLog
    static final MethodHandle HLL_ADD = h("rbx_hll_add_multi_n", JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS, ADDRESS, ADDRESS);
    static final MethodHandle HLL_COUNT = h("rbx_hll_count_n", JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS);
    static final MethodHandle HLL_MERGE = h("rbx_hll_merge_n", JAVA_INT, ADDRESS, NAME, ADDRESS, JAVA_INT);
    // asynchronous forms + futures
    static final MethodHandle HLL_ADD_ASYNC = h("rbx_hll_add_multi_async", JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS,
            ADDRESS, ADDRESS, ADDRESS, ADDRESS, ADDRESS);
    static final MethodHandle HLL_COUNT_ASYNC = h("rbx_hll_count_async", JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS,
            ADDRESS, ADDRESS, ADDRESS);
    static final MethodHandle HLL_MERGE_ASYNC = h("rbx_hll_merge_async", JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_INT,
            ADDRESS, ADDRESS, ADDRESS);
    static final MethodHandle FUTURE_WAIT = h("rbx_future_wait", JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS);
    static final MethodHandle FUTURE_FREE = h("rbx_future_free", JAVA_INT, ADDRESS);

    /** Maps the status codes of include/rbx.h to the exceptions the reference throws. */
    static RuntimeException error(int rc, String msg) {
        return switch (rc) {
            case -1 -> new IllegalArgumentException(msg);                 // RBX_E_ILLEGAL_ARGUMENT
            case -2 -> new IllegalStateException(msg);                    // "Bloom filter is not initialized!"
            case -3, -5, -8, -9 -> new RedisException(msg);               // config changed / WRONGTYPE / no such key / ERR
            case -4 -> new ArithmeticException(msg);                      // "/ by zero" (empty collection)
            default -> new IllegalStateException("rbx error " + rc + ": " + msg);
        };
    }

    static String lastError() {
        try { return ((MemorySegment) LAST_ERROR.invokeExact()).reinterpret(4096).getString(0); }
        catch (Throwable t) { return "?"; }
    }

    static void check(int rc) {
        if (rc != 0) throw error(rc, lastError());
    }

    static RuntimeException rethrow(Throwable t) {
        return t instanceof RuntimeException r ? r : new IllegalStateException(t);
    }

    /** struct rbx_name for a Java String key (Redisson encodes key names as UTF-8). */
    static MemorySegment name(Arena a, String s) {
        byte[] b = s.getBytes(java.nio.charset.StandardCharsets.UTF_8);
        MemorySegment n = a.allocate(NAME);
        n.set(ADDRESS, NAME_BYTES, a.allocateFrom(JAVA_BYTE, b.length == 0 ? new byte[1] : b));
        n.set(JAVA_LONG, NAME_LEN, b.length);
        return n;
    }

    static MemorySegment names(Arena a, String... s) {
        MemorySegment arr = a.allocate(NAME, Math.max(1, s.length));
        for (int i = 0; i < s.length; i++) MemorySegment.copy(name(a, s[i]), 0, arr, i * NAME_SIZE, NAME_SIZE);
        return arr;
    }

    /** Packs codec output into one off-heap arena: bytes + offsets[n+1] (struct rbx_keys). */
    static MemorySegment keys(Arena a, List<byte[]> enc) {
        long total = 0;
        for (byte[] b : enc) total += b.length;
        MemorySegment bytes = a.allocate(Math.max(total, 1));
        MemorySegment offs = a.allocate(JAVA_LONG, enc.size() + 1);
        long o = 0;
        for (int i = 0; i < enc.size(); i++) {
            offs.setAtIndex(JAVA_LONG, i, o);
            MemorySegment.copy(MemorySegment.ofArray(enc.get(i)), 0, bytes, o, enc.get(i).length);
            o += enc.get(i).length;
        }
        offs.setAtIndex(JAVA_LONG, enc.size(), o);
        MemorySegment k = a.allocate(KEYS);
        k.set(ADDRESS, KEYS_BYTES, bytes);
        k.set(ADDRESS, KEYS_OFFSETS, offs);
        k.set(JAVA_LONG, KEYS_STRIDE, 0L);
        k.set(JAVA_LONG, KEYS_N, (long) enc.size());
        return k;
    }

    // ---- completion upcall: void cb(void *user, int rc) ------------------------------------
    // The library calls it on the context's executor thread; `user` is a ticket into PENDING.
    record Pending(CompletableFuture<Object> cf, Arena arena, java.util.function.Supplier<Object> result) {}
    static final Map<Long, Pending> PENDING = new ConcurrentHashMap<>();
    static final AtomicLong TICKETS = new AtomicLong();
    static final MemorySegment CALLBACK;
    static {
        try {
            MethodHandle done = MethodHandles.lookup().findStatic(Rbx.class, "onDone",
                    MethodType.methodType(void.class, MemorySegment.class, int.class));
            CALLBACK = L.upcallStub(done, FunctionDescriptor.ofVoid(ADDRESS, JAVA_INT), Arena.global());
        } catch (ReflectiveOperationException e) { throw new ExceptionInInitializerError(e); }
    }

    static void onDone(MemorySegment user, int rc) {
        Pending p = PENDING.remove(user.address());
        if (p == null) return;
        try {
            if (rc == 0) p.cf().complete(p.result().get());
            else p.cf().completeExceptionally(error(rc, "async call failed (rbx code " + rc + ")"));
        } finally {
            p.arena().close();  // buffers the call read / wrote: valid until now
        }
    }

    /** Registers a pending call: returns the `user` ticket and the future the upcall completes. */
    @SuppressWarnings("unchecked")
    static <R> CompletableFuture<R> pending(Arena shared, java.util.function.Supplier<Object> result, long[] ticketOut) {
        long t = TICKETS.incrementAndGet();
        CompletableFuture<Object> cf = new CompletableFuture<>();
        PENDING.put(t, new Pending(cf, shared, result));
        ticketOut[0] = t;
        return (CompletableFuture<R>) (CompletableFuture<?>) cf;
    }
}
