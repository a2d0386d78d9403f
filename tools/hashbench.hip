// hashbench.hip -- standalone VALU-cost probe for the hash stage (not part of librbx.so).
//
//   hipcc -O3 --offload-arch=gfx950 -I redisson_amd/csrc tools/hashbench.hip -o tools/_build/hashbench
//   tools/_build/hashbench [nkeys]          -> one JSON line per measurement on stdout
//
// Measures, on nkeys random 32-byte keys resident in HBM (C2's key shape):
//   - the key stream alone (16-byte nontemporal loads, xor-reduced),
//   - HighwayHash128 of every key with the shipped rbx::hh128_fixed<32> and with candidate
//     legacy formulation (results must match the shipped hash bit for bit; a mismatch exits 1),
//   - hash + the 7 Bloom indexes (mod 2^32 and mod 95,850,583),
// plus instruction-issue rates of the VALU instructions the hash compiles to.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "rbx_device.h"

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(2);                                                                           \
        }                                                                                      \
    } while (0)

using namespace rbx;

__global__ void k_fill(uint32_t *p, uint64_t nwords, uint64_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t x = (i + 1) * 0x9e3779b97f4a7c15ULL ^ seed;
        x ^= x >> 31; x *= 0xbf58476d1ce4e5b9ULL; x ^= x >> 29; x *= 0x94d049bb133111ebULL; x ^= x >> 32;
        p[i] = (uint32_t)x;
    }
}

// The r01-r02 formulation of the same hash (64-bit `hi << 32 | lo` joins, swap32c operands),
// kept here as the A/B baseline of the shipped rbx::hh128_fixed.
namespace legacy {
__device__ __forceinline__ uint64_t j2(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
__device__ __forceinline__ uint64_t z0(uint64_t b, uint64_t a) {
    const uint32_t al = (uint32_t)a, ah = (uint32_t)(a >> 32), bh = (uint32_t)(b >> 32);
    const uint32_t t = perm_b32(bh, al, 0x0C020403u);
    return j2(perm_b32(ah, t, 0x05020100u), perm_b32(bh, al, 0x00070106u));
}
__device__ __forceinline__ uint64_t z1(uint64_t b, uint64_t a) {
    const uint32_t ah = (uint32_t)(a >> 32), bl = (uint32_t)b, bh = (uint32_t)(b >> 32);
    const uint32_t t = perm_b32(ah, bl, 0x0C020403u);
    return j2(perm_b32(bh, t, 0x05020100u), perm_b32(ah, bl, 0x07000601u));
}
__device__ __forceinline__ void upd(HH &s, uint64_t a0, uint64_t a1, uint64_t a2, uint64_t a3) {
    s.v1[0] += s.mul0[0] + a0;
    s.v1[1] += s.mul0[1] + a1;
    s.v1[2] += s.mul0[2] + a2;
    s.v1[3] += s.mul0[3] + a3;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        s.mul0[i] ^= mul32x32(s.v1[i], s.v0[i]);
        s.v0[i] += s.mul1[i];
        s.mul1[i] ^= mul32x32(s.v0[i], s.v1[i]);
    }
    s.v0[0] += z0(s.v1[1], s.v1[0]);
    s.v0[1] += z1(s.v1[1], s.v1[0]);
    s.v0[2] += z0(s.v1[3], s.v1[2]);
    s.v0[3] += z1(s.v1[3], s.v1[2]);
    s.v1[0] += z0(s.v0[1], s.v0[0]);
    s.v1[1] += z1(s.v0[1], s.v0[0]);
    s.v1[2] += z0(s.v0[3], s.v0[2]);
    s.v1[3] += z1(s.v0[3], s.v0[2]);
}
__device__ __forceinline__ void hash32(const uint8_t *p, uint64_t &h1, uint64_t &h2) {
    HH s;
    hh_reset(s);
    const uint4 x0 = ld_nt16(p), x1 = ld_nt16(p + 16);
    upd(s, j2(x0.x, x0.y), j2(x0.z, x0.w), j2(x1.x, x1.y), j2(x1.z, x1.w));
#pragma unroll
    for (int r = 0; r < 6; ++r) upd(s, swap32c(s.v0[2]), swap32c(s.v0[3]), swap32c(s.v0[0]), swap32c(s.v0[1]));
    h1 = s.v0[0] + s.mul0[0] + s.v1[2] + s.mul1[2];
    h2 = s.v0[1] + s.mul0[1] + s.v1[3] + s.mul1[3];
}
}  // namespace legacy

// candidate: r02o experiment "V3" exactly as first measured (whole-lane first step, then halves)
namespace v3 {
__device__ __forceinline__ void upd_tail(HH &s) { hh_update_tail(s); }
__device__ __forceinline__ void hash32(const uint8_t *p, uint64_t &h1, uint64_t &h2) {
    HH s;
    hh_reset(s);
    const uint4 x0 = ld_nt16(p), x1 = ld_nt16(p + 16);
    hh_update(s, w2(x0.x, x0.y), w2(x0.z, x0.w), w2(x1.x, x1.y), w2(x1.z, x1.w));
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        const int src[4] = {2, 3, 0, 1};
        uint64_t t[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) t[i] = s.v1[i] + s.mul0[i];
#pragma unroll
        for (int i = 0; i < 4; ++i) s.v1[i] = add_halves(t[i], (uint32_t)(s.v0[src[i]] >> 32), (uint32_t)s.v0[src[i]]);
        upd_tail(s);
    }
    h1 = s.v0[0] + s.mul0[0] + s.v1[2] + s.mul1[2];
    h2 = s.v0[1] + s.mul0[1] + s.v1[3] + s.mul1[3];
}
}  // namespace v3

// V = 0: the shipped hash; V = 1: the legacy formulation; V = 2: candidate
template <int V>
__device__ __forceinline__ void hash32(const uint8_t *p, uint64_t &h1, uint64_t &h2) {
    if constexpr (V == 0) hh128_fixed<32>(p, h1, h2);
    else if constexpr (V == 1) legacy::hash32(p, h1, h2);
    else v3::hash32(p, h1, h2);
}

// MODE 0: key stream only; 1: hash; 2: hash + 7 indexes mod 2^32; 3: hash + 7 indexes mod 95,850,583
template <int V, int MODE>
__global__ __launch_bounds__(256) void k_hash(const uint8_t *keys, uint64_t n, ModParams mp, uint64_t *out) {
    uint64_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint8_t *p = keys + i * 32;
        if constexpr (MODE == 0) {
            const uint4 a = ld_nt16(p), b = ld_nt16(p + 16);
            acc ^= w2(a.x ^ b.x, a.y ^ b.y) + w2(a.z ^ b.z, a.w ^ b.w);
        } else {
            uint64_t h1, h2;
            hash32<V>(p, h1, h2);
            if constexpr (MODE == 1) {
                acc ^= h1 + 3 * h2;
            } else {
                uint64_t h = h1;
#pragma unroll
                for (int j = 0; j < 7; ++j) {
                    acc += mod63(h & 0x7fffffffffffffffULL, mp);
                    h += (j & 1) ? h1 : h2;
                }
            }
        }
    }
    out[blockIdx.x * (uint64_t)blockDim.x + threadIdx.x] = acc;
}

// Instruction issue probes: 8 independent chains per lane, 64 rounds per loop trip.
template <int OP>
__global__ __launch_bounds__(256) void k_ipt(uint32_t iters, uint32_t seed, uint64_t *out) {
    uint64_t a[8];
    uint32_t b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = (uint64_t)(threadIdx.x + j * 977 + seed) * 0x9e3779b97f4a7c15ULL;
        b[j] = (uint32_t)(a[j] >> 17) | 1u;
    }
    const uint32_t sel = 0x05020100u + seed;
    for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(b[j]) : "v"(b[(j + 1) & 7]));
                if constexpr (OP == 1) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]));
                if constexpr (OP == 2) {
                    uint64_t c;
                    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(a[j]), "=s"(c) : "v"(b[j]), "v"(b[(j + 1) & 7]));
                }
                if constexpr (OP == 3) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(b[j]) : "v"(b[(j + 1) & 7]), "s"(sel));
                if constexpr (OP == 4) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(b[j]) : "v"(b[(j + 1) & 7]));
                if constexpr (OP == 5) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(b[j]) : "v"(b[(j + 1) & 7]));
                if constexpr (OP == 6) {
                    uint32_t lo = (uint32_t)a[j], hi = (uint32_t)(a[j] >> 32);
                    asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc"
                                 : "+v"(lo), "+v"(hi) : "v"(b[j]), "v"(b[(j + 1) & 7]) : "vcc");
                    a[j] = ((uint64_t)hi << 32) | lo;
                }
                if constexpr (OP == 7) asm volatile("v_mov_b32 %0, %1" : "=v"(b[j]) : "v"(b[(j + 3) & 7]));
                if constexpr (OP == 8) asm volatile("v_add_u32 %0, %0, %1" : "+v"(b[j]) : "v"(b[(j + 1) & 7]));
                if constexpr (OP == 9) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(b[j]) : "v"(b[(j + 1) & 7]));
                if constexpr (OP == 10) asm volatile("v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]" : "+v"(a[j]));
                if constexpr (OP == 11) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(b[j]) : "v"(b[(j + 1) & 7]), "v"(b[(j + 2) & 7]));
            }
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] + b[j];
    out[blockIdx.x * (uint64_t)blockDim.x + threadIdx.x] = s;
}

static float time_ms(hipEvent_t e0, hipEvent_t e1) {
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
}

template <class F> static float best_of(int reps, F launch) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, 0));
        launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        const float t = time_ms(e0, e1);
        if (t < best) best = t;
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return best;
}

static uint64_t checksum(const uint64_t *d, size_t n) {
    std::vector<uint64_t> h(n);
    CK(hipMemcpy(h.data(), d, n * 8, hipMemcpyDeviceToHost));
    uint64_t s = 0;
    for (size_t i = 0; i < n; ++i) s = s * 0x100000001b3ULL + h[i];
    return s;
}

template <int V, int MODE> static void run_hash(const uint8_t *keys, uint64_t n, const ModParams &mp, uint64_t *out,
                                               unsigned grid, uint64_t ref, uint64_t *cs) {
    const float ms = best_of(5, [&] { hipLaunchKernelGGL((k_hash<V, MODE>), dim3(grid), dim3(256), 0, 0, keys, n, mp, out); });
    const uint64_t c = checksum(out, (size_t)grid * 256);
    if (cs) *cs = c;
    const bool ok = ref == 0 || c == ref;
    printf("{\"probe\": \"hash\", \"variant\": %d, \"mode\": %d, \"keys\": %llu, \"grid\": %u, \"ms\": %.4f, "
           "\"keys_per_s\": %.4e, \"checksum_ok\": %s}\n",
           V, MODE, (unsigned long long)n, grid, ms, n / (ms * 1e-3), ok ? "true" : "false");
    fflush(stdout);
    if (!ok) exit(1);
}

template <int OP> static void run_ipt(uint64_t *out, const char *name) {
    const unsigned grid = 256 * 8;  // 8 blocks of 4 waves per CU: 8 waves per SIMD
    const uint32_t iters = 4096;
    const float ms = best_of(3, [&] { hipLaunchKernelGGL((k_ipt<OP>), dim3(grid), dim3(256), 0, 0, iters, 1u, out); });
    const double winst = (double)grid * 4 * iters * 64;  // wave-instructions
    const double simd_cyc = ms * 1e-3 * 1024 * 2.4e9;      // SIMD-cycles at 2.4 GHz
    const int per = (OP == 6) ? 2 : 1;
    printf("{\"probe\": \"ipt\", \"op\": \"%s\", \"ms\": %.4f, \"cyc_per_wave_inst_at_2p4GHz\": %.2f}\n", name, ms,
           simd_cyc / (winst * per));
    fflush(stdout);
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 100000000ULL;
    uint8_t *keys;
    uint64_t *out;
    CK(hipMalloc(&keys, n * 32));
    const unsigned maxgrid = 256 * 32;
    CK(hipMalloc(&out, (size_t)maxgrid * 256 * 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)keys, n * 8, 0x1234ULL);
    CK(hipDeviceSynchronize());
    const ModParams mp32 = make_mod_params(1ULL << 32), mpc1 = make_mod_params(95850583ULL);
    uint64_t c1 = 0, c2 = 0, c3 = 0;
    for (unsigned grid : {2048u, 8192u}) {
        run_hash<0, 0>(keys, n, mp32, out, grid, 0, nullptr);
        run_hash<0, 1>(keys, n, mp32, out, grid, 0, &c1);
        run_hash<1, 1>(keys, n, mp32, out, grid, c1, nullptr);
        run_hash<2, 1>(keys, n, mp32, out, grid, c1, nullptr);
        run_hash<0, 1>(keys, n, mp32, out, grid, c1, nullptr);
        run_hash<0, 2>(keys, n, mp32, out, grid, 0, &c2);
        run_hash<1, 2>(keys, n, mp32, out, grid, c2, nullptr);
        run_hash<0, 3>(keys, n, mpc1, out, grid, 0, &c3);
        run_hash<1, 3>(keys, n, mpc1, out, grid, c3, nullptr);
    }
    run_ipt<0>(out, "v_xor_b32");
    run_ipt<8>(out, "v_add_u32");
    run_ipt<7>(out, "v_mov_b32");
    run_ipt<1>(out, "v_lshl_add_u64");
    run_ipt<2>(out, "v_mad_u64_u32");
    run_ipt<3>(out, "v_perm_b32");
    run_ipt<4>(out, "v_mul_lo_u32");
    run_ipt<5>(out, "v_mul_hi_u32");
    run_ipt<6>(out, "v_add_co+v_addc_co (per inst)");
    run_ipt<9>(out, "v_mul_u32_u24");
    run_ipt<10>(out, "v_pk_mov_b32");
    run_ipt<11>(out, "v_bitop3_b32");
    CK(hipFree(keys));
    CK(hipFree(out));
    return 0;
}
