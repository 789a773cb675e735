// calib_fetch.hip — calibrates the HBM byte counters (FETCH_SIZE, WRITE_SIZE,
// TCC_EA0_RDREQ_{32B,64B,128B}) on the access patterns of this repository's
// kernels, with known byte counts, on buffers far larger than the 256 MiB
// last-level cache.  MI355X_MICROARCH.md calibrates FETCH_SIZE only for wide
// streaming reads ("report exactly 1/2 ... double it"); the wavefront kernels
// also gather 48-B ray records and 32-B path records by slot and scatter
// 24-B sample records, whose counter factors this tool measures.
//
//   build: hipcc -O3 --offload-arch=gfx950 -o calib_fetch tools/calib_fetch.hip
//   run:   rocprofv3 --pmc FETCH_SIZE -- ./calib_fetch      (one counter set per run)
//
// Each pattern is one kernel launch (name = pattern), preceded by a cache
// flush kernel; the program prints each pattern's algorithmic bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

struct alignas(16) R48 { double a[6]; };
struct alignas(16) R32 { double a[4]; };

constexpr uint32_t kN = 1u << 25;          // records per pattern (48 B x 32M = 1.5 GiB)
__device__ __forceinline__ uint32_t scatter(uint32_t i) { return (i * 2654435761u) & (kN - 1); }   // bijection on [0, kN)
// ascending with gaps: ~70 % of the slots, as a material queue sees its rays
__device__ __forceinline__ uint32_t gapped(uint32_t i) { return (uint32_t)(((uint64_t)i * 10u) / 7u); }

__global__ void seq16(const uint4* __restrict__ in, double* __restrict__ sink) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const uint4 v = in[i];
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x7FFFFFFFu) sink[0] = 1.0;
}
__global__ void seq48(const R48* __restrict__ in, double* __restrict__ sink) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const R48 r = in[i];
    if (r.a[0] + r.a[1] + r.a[2] + r.a[3] + r.a[4] + r.a[5] == 12345.0) sink[0] = 1.0;
}
__global__ void gather48(const R48* __restrict__ in, double* __restrict__ sink) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const R48 r = in[scatter(i)];
    if (r.a[0] + r.a[1] + r.a[2] + r.a[3] + r.a[4] + r.a[5] == 12345.0) sink[0] = 1.0;
}
__global__ void gapped48(const R48* __restrict__ in, double* __restrict__ sink, uint32_t n) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const R48 r = in[gapped(i)];
    if (r.a[0] + r.a[1] + r.a[2] + r.a[3] + r.a[4] + r.a[5] == 12345.0) sink[0] = 1.0;
}
__global__ void gather32(const R32* __restrict__ in, double* __restrict__ sink) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const R32 r = in[scatter(i)];
    if (r.a[0] + r.a[1] + r.a[2] + r.a[3] == 12345.0) sink[0] = 1.0;
}
__global__ void gapped32(const R32* __restrict__ in, double* __restrict__ sink, uint32_t n) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const R32 r = in[gapped(i)];
    if (r.a[0] + r.a[1] + r.a[2] + r.a[3] == 12345.0) sink[0] = 1.0;
}
__global__ void wseq16(uint4* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    out[i] = make_uint4(i, i + 1, i + 2, i + 3);
}
__global__ void wseq48(R48* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const double v = (double)i;
    out[i] = R48{{v, v, v, v, v, v}};
}
__global__ void wseq32(R32* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const double v = (double)i;
    out[i] = R32{{v, v, v, v}};
}
__global__ void wscatter24(double* __restrict__ out) {       // one rgb sample record per scattered work id
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    double* o = out + 3u * (size_t)scatter(i);
    const double v = (double)i;
    o[0] = v; o[1] = v; o[2] = v;
}
__global__ void flush(const uint4* __restrict__ in, size_t n, double* __restrict__ sink) {   // evict the caches
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += (size_t)gridDim.x * 256u) acc ^= in[i].x;
    if (acc == 0x7FFFFFFFu) sink[1] = 1.0;
}

int main() {
    const size_t bytes = (size_t)kN * sizeof(R48);
    void *a = nullptr, *b = nullptr, *f = nullptr;
    double* sink = nullptr;
    const size_t fbytes = (size_t)1 << 30;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&f, fbytes));
    CK(hipMalloc((void**)&sink, 64));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 0, bytes));
    CK(hipMemset(f, 2, fbytes));
    const dim3 g(kN / 256), blk(256);
    const uint32_t ngap = (uint32_t)(((uint64_t)kN * 7u) / 10u) - 1u;
    auto fl = [&] { hipLaunchKernelGGL(flush, dim3(4096), blk, 0, 0, (const uint4*)f, fbytes / 16, sink); };
    struct P { const char* name; double algo_bytes; };
    const P pats[] = {{"seq16", 16.0 * kN}, {"seq48", 48.0 * kN}, {"gather48", 48.0 * kN}, {"gapped48", 48.0 * ngap},
                      {"gather32", 32.0 * kN}, {"gapped32", 32.0 * ngap}, {"wseq16", 16.0 * kN},
                      {"wseq48", 48.0 * kN}, {"wseq32", 32.0 * kN}, {"wscatter24", 24.0 * kN}};
    fl(); hipLaunchKernelGGL(seq16, g, blk, 0, 0, (const uint4*)a, sink);
    fl(); hipLaunchKernelGGL(seq48, g, blk, 0, 0, (const R48*)a, sink);
    fl(); hipLaunchKernelGGL(gather48, g, blk, 0, 0, (const R48*)a, sink);
    fl(); hipLaunchKernelGGL(gapped48, dim3((ngap + 255) / 256), blk, 0, 0, (const R48*)a, sink, ngap);
    fl(); hipLaunchKernelGGL(gather32, g, blk, 0, 0, (const R32*)a, sink);
    fl(); hipLaunchKernelGGL(gapped32, dim3((ngap + 255) / 256), blk, 0, 0, (const R32*)a, sink, ngap);
    fl(); hipLaunchKernelGGL(wseq16, g, blk, 0, 0, (uint4*)b);
    fl(); hipLaunchKernelGGL(wseq48, g, blk, 0, 0, (R48*)b);
    fl(); hipLaunchKernelGGL(wseq32, g, blk, 0, 0, (R32*)b);
    fl(); hipLaunchKernelGGL(wscatter24, g, blk, 0, 0, (double*)b);
    CK(hipDeviceSynchronize());
    for (const P& p : pats) std::printf("{\"pattern\": \"%s\", \"algo_bytes\": %.0f}\n", p.name, p.algo_bytes);
    CK(hipFree(a)); CK(hipFree(b)); CK(hipFree(f)); CK(hipFree(sink));
    return 0;
}
