// fetch_calib.hip — what rocprofv3's FETCH_SIZE reports for the access widths of the mesh kernels
// (tools only).  MI355X_MICROARCH.md: on gfx950 FETCH_SIZE is exactly 1/2 of the bytes of a wide
// coalesced streaming read (128-B requests tallied at 64 B); other widths are uncalibrated.  The
// traversal kernels read 64-B BVH pair records and 16 / 32-B queue words at scattered slots, so
// their "2 x FETCH_SIZE" traffic needs this calibration: each kernel below reads a known byte count
// in one pattern over a 1 GiB buffer (past the 256 MB Infinity Cache):
//   k_stream   16 B per lane, coalesced (the guide's calibrated case)
//   k_rand16   one float4 per lane at a random 16-B slot
//   k_rand32   two float4 (32 B) per lane at a random 32-B slot
//   k_rand64   four float4 (64 B, one BVH pair record) per lane at a random 64-B slot
//   k_rand128  eight float4 (128 B) per lane at a random 128-B slot
// every kernel reading 256 MiB.  Run under `rocprofv3 --kernel-trace --pmc FETCH_SIZE`; the program
// prints each kernel's algorithmic read bytes.
//
//   hipcc --offload-arch=gfx950 -O3 -o project3-cuda-path-tracer-2025_amd/build/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                        \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__device__ __forceinline__ unsigned mix(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(256) void k_stream(const float4* __restrict__ in, float* __restrict__ out, unsigned n) {
    const unsigned i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const float4 v = in[i];
    if (v.x == 1.2345f) out[i & 1023] = v.y + v.z + v.w;   // never true: keeps the load
}
template <int F4>   // F4 float4 per lane, at a random slot of F4 float4
__global__ __launch_bounds__(256) void k_rand(const float4* __restrict__ in, float* __restrict__ out, unsigned lanes,
                                              unsigned slots) {
    const unsigned i = blockIdx.x * 256u + threadIdx.x;
    if (i >= lanes) return;
    const size_t s = (size_t)(mix(i * 2654435761u + 12345u) % slots) * F4;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < F4; ++k) {
        const float4 v = in[s + k];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1.2345f) out[i & 1023] = acc;
}

int main() {
    const size_t buf = (size_t)1 << 30;                  // 1 GiB of float4
    const size_t n4 = buf / 16;
    const size_t read = (size_t)256 << 20;               // 256 MiB read by every kernel
    float4* in;
    float* out;
    CHK(hipMalloc(&in, buf));
    CHK(hipMalloc(&out, 4096 * sizeof(float)));
    CHK(hipMemset(in, 0, buf));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    auto run = [&](const char* name, auto launch) {
        for (int rep = 0; rep < 3; ++rep) {
            CHK(hipEventRecord(a));
            launch();
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms = 0.f;
            CHK(hipEventElapsedTime(&ms, a, b));
            printf("{\"kernel\": \"%s\", \"rep\": %d, \"read_bytes\": %zu, \"ms\": %.4f, \"GBps\": %.1f}\n", name, rep, read, ms,
                   read / (ms * 1e-3) / 1e9);
        }
    };
    const unsigned ls = (unsigned)(read / 16);
    run("k_stream", [&] { hipLaunchKernelGGL(k_stream, dim3((ls + 255) / 256), dim3(256), 0, 0, in, out, ls); });
    run("k_rand16", [&] {
        hipLaunchKernelGGL(k_rand<1>, dim3((ls + 255) / 256), dim3(256), 0, 0, in, out, ls, (unsigned)(n4 / 1));
    });
    run("k_rand32", [&] {
        const unsigned l = ls / 2;
        hipLaunchKernelGGL(k_rand<2>, dim3((l + 255) / 256), dim3(256), 0, 0, in, out, l, (unsigned)(n4 / 2));
    });
    run("k_rand64", [&] {
        const unsigned l = ls / 4;
        hipLaunchKernelGGL(k_rand<4>, dim3((l + 255) / 256), dim3(256), 0, 0, in, out, l, (unsigned)(n4 / 4));
    });
    run("k_rand128", [&] {
        const unsigned l = ls / 8;
        hipLaunchKernelGGL(k_rand<8>, dim3((l + 255) / 256), dim3(256), 0, 0, in, out, l, (unsigned)(n4 / 8));
    });
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    CHK(hipFree(in));
    CHK(hipFree(out));
    return 0;
}
