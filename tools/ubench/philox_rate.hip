// Philox4x32-10 issue cost on one SIMD (dev microbenchmark for the dropout design).
// Every thread runs NCALL Philox calls on its own counter; one wave per SIMD (256 threads / block,
// one block per CU). Wave 0 of each block stamps s_memtime / s_memrealtime around its loop.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/philox_rate.hip -o /tmp/philox_rate && /tmp/philox_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[1] = (uint32_t)p1; c[3] = (uint32_t)p0; c[0] = n0; c[2] = n2;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

template <int NCALL>
__global__ __launch_bounds__(256) void k_philox(uint32_t* out, uint64_t* stamps, uint32_t seed_lo, uint32_t seed_hi) {
    uint64_t t0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
    uint32_t tid = blockIdx.x * 256 + threadIdx.x;
    for (int i = 0; i < NCALL; i += 2) {
        uint32_t a[4] = {tid, (uint32_t)i, 7u, 0u}, b[4] = {tid, (uint32_t)i + 1, 7u, 0u};
        philox(a, seed_lo, seed_hi);
        philox(b, seed_lo, seed_hi);
        acc ^= a[0] ^ a[1] ^ a[2] ^ a[3] ^ b[0] ^ b[1] ^ b[2] ^ b[3];
    }
    uint64_t t1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();
    out[tid] = acc;
    if (threadIdx.x == 0) { stamps[2 * blockIdx.x] = t1 - t0; stamps[2 * blockIdx.x + 1] = r1 - r0; }
}

int main() {
    const int nb = 256, ncall = 4096;
    uint32_t* out; uint64_t* st;
    CHK(hipMalloc(&out, nb * 256 * 4)); CHK(hipMalloc(&st, nb * 16));
    for (int it = 0; it < 3; ++it) {
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        k_philox<ncall><<<nb, 256>>>(out, st, 0x1234u, 0x5678u);
        hipEventRecord(e1); CHK(hipEventSynchronize(e1));
        float ms; hipEventElapsedTime(&ms, e0, e1);
        uint64_t h[2 * nb]; CHK(hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost));
        double cyc = 0, rt = 0; for (int b = 0; b < nb; ++b) { cyc += h[2 * b]; rt += h[2 * b + 1]; }
        cyc /= nb; rt /= nb;
        printf("launch %.3f ms; wave loop %.0f cycles, clock %.2f GHz; %.1f cycles per Philox call per wave "
               "(one wave per SIMD)\n", ms, cyc, cyc / rt * 0.1, cyc / ncall);
    }
    return 0;
}
