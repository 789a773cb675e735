#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int V>
__device__ __forceinline__ void philox(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint32_t lo0, hi0, lo1, hi1;
        if (V == 0) {
            lo0 = 0xD2511F53u * c0; hi0 = __umulhi(0xD2511F53u, c0);
            lo1 = 0xCD9E8D57u * c2; hi1 = __umulhi(0xCD9E8D57u, c2);
        } else {
            const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
            lo0 = (uint32_t)p0; hi0 = (uint32_t)(p0 >> 32); lo1 = (uint32_t)p1; hi1 = (uint32_t)(p1 >> 32);
        }
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
}
template <int V>
__global__ void k(uint32_t* out, int iters) {
    uint32_t a = blockIdx.x * 256 + threadIdx.x, b = 1, c = 2, d = 3, x = 0;
    for (int i = 0; i < iters; ++i) { uint32_t c0 = a + i, c1 = b, c2 = c, c3 = d; philox<V>(c0, c1, c2, c3, 7, 9); x ^= c0 ^ c1 ^ c2 ^ c3; }
    out[blockIdx.x * 256 + threadIdx.x] = x;
}
int main() {
    uint32_t* o; hipMalloc(&o, 4 << 22);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) for (int V = 0; V < 2; ++V) {
        hipEventRecord(e0);
        if (V == 0) hipLaunchKernelGGL(k<0>, dim3(16384), dim3(256), 0, 0, o, 256);
        else hipLaunchKernelGGL(k<1>, dim3(16384), dim3(256), 0, 0, o, 256);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("V%d %.3f ms  %.2f Gblocks/s\n", V, ms, 16384.0 * 256 * 256 / ms / 1e6);
    }
    uint32_t h[4]; hipMemcpy(h, o, 16, hipMemcpyDeviceToHost); printf("%u\n", h[0]);
}
