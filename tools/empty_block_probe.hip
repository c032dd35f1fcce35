// empty_block_probe.hip — what a block that exits at once costs on gfx950 (tools only).
//
// k_bounce / k_bvh_bounce are captured with the pass's full grid (one block per 256 paths of
// bounce 0); in the late bounces most blocks find `block_start >= n` and return.  This probe
// times launches whose blocks all return after reading the live count, by grid size and by the
// dynamic LDS the launch asks for (k_bounce: ~20 KB), against a grid of the same kernel where
// every block does a little work, so the per-empty-block price can be read off.
//
//   hipcc --offload-arch=gfx950 -O3 -o build/empty_block_probe tools/empty_block_probe.hip && ./build/empty_block_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

__global__ __launch_bounds__(256) void k_empty(const int* __restrict__ ctl, float* __restrict__ out) {
    extern __shared__ float s[];
    int n = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) n += ctl[k * 32];   // the 8 segment counters, like k_bounce
    const int block_start = blockIdx.x * 256;
    if (block_start >= n) return;
    const int gid = block_start + threadIdx.x;
    s[threadIdx.x] = (float)gid;
    __syncthreads();
    if (gid < n) out[gid] = s[255 - threadIdx.x];
}

int main() {
    int* d_ctl;
    float* d_out;
    CHK(hipMalloc(&d_ctl, 8 * 32 * sizeof(int)));
    CHK(hipMalloc(&d_out, 64 << 20));
    hipStream_t st;
    CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const int grids[] = {1024, 4096, 16384, 50000, 100000};
    const size_t ldss[] = {0, 20480};
    const int lives[] = {0, 256 * 2048};
    for (int live : lives) {
        std::vector<int> h(8 * 32, 0);
        h[0] = live;
        CHK(hipMemcpy(d_ctl, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice));
        for (size_t lds : ldss)
            for (int g : grids) {
                for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), lds, st, d_ctl, d_out);
                std::vector<float> ts;
                for (int r = 0; r < 20; ++r) {
                    CHK(hipEventRecord(a, st));
                    hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), lds, st, d_ctl, d_out);
                    CHK(hipEventRecord(b, st));
                    CHK(hipEventSynchronize(b));
                    float ms = 0;
                    CHK(hipEventElapsedTime(&ms, a, b));
                    ts.push_back(ms * 1000.f);
                }
                std::sort(ts.begin(), ts.end());
                printf("{\"live_paths\": %d, \"grid\": %d, \"lds\": %zu, \"us_median\": %.2f, \"us_min\": %.2f}\n", live,
                       g, lds, ts[ts.size() / 2], ts[0]);
            }
    }
    return 0;
}
