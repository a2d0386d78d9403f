// syncbench: how a synchronous one-kernel call learns that its kernel is done.
//   hipcc --offload-arch=gfx950 -O2 -o tools/_build/syncbench tools/syncbench.hip && tools/_build/syncbench
// (a) launch + hipStreamSynchronize; (b) the kernel's last store is a flag in coherent pinned memory and the
// host spins on it; (c) launch + a 1-thread flag kernel + spin; (d) (a) with hipDeviceScheduleSpin.
// Median over 2000 calls of a one-wave kernel that reads one word of HBM and writes one byte to the host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

__global__ void k_work(const unsigned *src, unsigned char *out, unsigned *flag, unsigned seq) {
    if (threadIdx.x != 0) return;
    out[0] = (unsigned char)(src[seq & 1023] & 1u);
    if (flag) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_flag(unsigned *flag, unsigned seq) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void spin(volatile unsigned *f, unsigned seq, hipStream_t st) {
    const double t0 = now_us();
    while (__atomic_load_n(f, __ATOMIC_ACQUIRE) != seq)
        if (now_us() - t0 > 100000) {  // a fault: let the runtime report it
            CK(hipStreamSynchronize(st));
            fprintf(stderr, "flag never came\n");
            exit(1);
        }
}

int main(int argc, char **argv) {
    const int mode_spin = argc > 1 ? atoi(argv[1]) : 0;
    if (mode_spin) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    unsigned *src;
    CK(hipMalloc(&src, 4096));
    CK(hipMemset(src, 0x5a, 4096));
    unsigned char *hb;
    CK(hipHostMalloc((void **)&hb, 4096, hipHostMallocCoherent | hipHostMallocMapped));
    unsigned char *db;
    CK(hipHostGetDevicePointer((void **)&db, hb, 0));
    unsigned *hflag = (unsigned *)(hb + 64), *dflag = (unsigned *)(db + 64);
    *hflag = 0;
    const char *names[3] = {"launch+hipStreamSynchronize", "kernel flag + host spin", "launch+flag kernel + spin"};
    unsigned seq = 1;
    for (int m = 0; m < 3; ++m) {
        std::vector<double> t;
        for (int i = 0; i < 2200; ++i, ++seq) {
            const double t0 = now_us();
            if (m == 0) {
                hipLaunchKernelGGL(k_work, dim3(1), dim3(64), 0, st, src, db, (unsigned *)nullptr, seq);
                CK(hipStreamSynchronize(st));
            } else if (m == 1) {
                hipLaunchKernelGGL(k_work, dim3(1), dim3(64), 0, st, src, db, dflag, seq);
                spin(hflag, seq, st);
            } else {
                hipLaunchKernelGGL(k_work, dim3(1), dim3(64), 0, st, src, db, (unsigned *)nullptr, seq);
                hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, st, dflag, seq);
                spin(hflag, seq, st);
            }
            if (i >= 200) t.push_back(now_us() - t0);
        }
        CK(hipStreamSynchronize(st));
        std::sort(t.begin(), t.end());
        printf("{\"bench\": \"syncbench\", \"schedule_spin\": %d, \"mode\": \"%s\", \"median_us\": %.2f, \"p10_us\": %.2f, "
               "\"p90_us\": %.2f}\n",
               mode_spin, names[m], t[t.size() / 2], t[t.size() / 10], t[t.size() * 9 / 10]);
    }
    CK(hipHostFree(hb));
    CK(hipFree(src));
    CK(hipStreamDestroy(st));
    return 0;
}
