// ta_probe.hip — what a divergent 64-B record fetch costs on gfx950 (tools only, not the product).
//
// k_bvh_bounce's inner step fetches one 64-B DevPair per lane with 4 dwordx4 loads, every
// lane from its own record (bunny: texture addresser 72 % busy, profiles/r04_instmix_ta_c4_bunny).
// This probe times dependent chains of random record fetches from an L2-resident table:
//   own   : each lane loads its own record, 4 x dwordx4 (the product's access)
//   coop  : the 4 lanes of a quad load the 4 records of the quad's rays together, one dwordx4
//           per lane per record (each load instruction touches 16 records, 4 lanes per record),
//           then exchange through LDS so every lane holds its own record (ds_write_b128 x 1,
//           ds_read_b128 x 4)
//   coopx : coop without the LDS exchange (the fetch alone)
// Records per second per variant, for table sizes like bunny's pairs (106 KB) and khaslana's.
//
//   hipcc --offload-arch=gfx950 -O3 -o build/ta_probe tools/ta_probe.hip && ./build/ta_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

constexpr int BLOCK = 256;

__device__ inline uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    return x;
}

// next record index from the fetched data (a dependent chain, like a traversal)
__device__ inline uint32_t next_idx(uint32_t idx, const float4& a, const float4& b, const float4& c,
                                    const float4& d, uint32_t n) {
    const uint32_t h = __float_as_uint(a.x) ^ __float_as_uint(b.y) ^ __float_as_uint(c.z) ^ __float_as_uint(d.w);
    return mix(h ^ idx) % n;
}

__global__ __launch_bounds__(BLOCK) void k_own(const float4* __restrict__ tab, uint32_t n, int steps,
                                                uint32_t* __restrict__ out) {
    const uint32_t gid = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t idx = mix(gid) % n;
    for (int s = 0; s < steps; ++s) {
        const float4* r = tab + 4 * (size_t)idx;
        const float4 a = r[0], b = r[1], c = r[2], d = r[3];
        idx = next_idx(idx, a, b, c, d, n);
    }
    out[gid] = idx;
}

template <bool XCHG>
__global__ __launch_bounds__(BLOCK) void k_coop(const float4* __restrict__ tab, uint32_t n, int steps,
                                                 uint32_t* __restrict__ out) {
    __shared__ float4 x[BLOCK][4];
    const uint32_t gid = blockIdx.x * BLOCK + threadIdx.x;
    const int lane = threadIdx.x & 63, q = lane & ~3, k = lane & 3;
    uint32_t idx = mix(gid) % n;
    for (int s = 0; s < steps; ++s) {
        float4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {   // record of ray q + j, chunk k
            const uint32_t rj = __shfl(idx, q + j, 64);
            v[j] = tab[4 * (size_t)rj + k];
        }
        float4 a, b, c, d;
        if (XCHG) {
#pragma unroll
            for (int j = 0; j < 4; ++j) x[(threadIdx.x & ~3) + j][k] = v[j];
            __builtin_amdgcn_wave_barrier();
            a = x[threadIdx.x][0];
            b = x[threadIdx.x][1];
            c = x[threadIdx.x][2];
            d = x[threadIdx.x][3];
            __builtin_amdgcn_wave_barrier();
        } else {   // the fetch alone: chain through the fetched chunks without exchanging them
            a = v[0];
            b = v[1];
            c = v[2];
            d = v[3];
        }
        idx = next_idx(idx, a, b, c, d, n);
    }
    out[gid] = idx;
}

int main(int argc, char** argv) {
    const int steps = 64;
    const int nblocks = 256 * 8 * 8;   // 8 blocks per CU x 8 rounds
    uint32_t* d_out;
    CHK(hipMalloc(&d_out, sizeof(uint32_t) * nblocks * BLOCK));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const size_t sizes[] = {106 * 1024, 1 << 20, 4 << 20};
    for (size_t bytes : sizes) {
        const uint32_t n = (uint32_t)(bytes / 64);
        std::vector<float> h(16 * (size_t)n);
        for (size_t i = 0; i < h.size(); ++i) h[i] = (float)(rand() & 0xffff);
        float4* d_tab;
        CHK(hipMalloc(&d_tab, 64 * (size_t)n));
        CHK(hipMemcpy(d_tab, h.data(), 64 * (size_t)n, hipMemcpyHostToDevice));
        for (int v = 0; v < 3; ++v) {
            float best = 1e30f;
            for (int rep = 0; rep < 5; ++rep) {
                CHK(hipEventRecord(e0));
                if (v == 0) hipLaunchKernelGGL(k_own, dim3(nblocks), dim3(BLOCK), 0, 0, d_tab, n, steps, d_out);
                if (v == 1) hipLaunchKernelGGL(k_coop<true>, dim3(nblocks), dim3(BLOCK), 0, 0, d_tab, n, steps, d_out);
                if (v == 2) hipLaunchKernelGGL(k_coop<false>, dim3(nblocks), dim3(BLOCK), 0, 0, d_tab, n, steps, d_out);
                CHK(hipEventRecord(e1));
                CHK(hipEventSynchronize(e1));
                float ms;
                CHK(hipEventElapsedTime(&ms, e0, e1));
                if (rep > 0 && ms < best) best = ms;
            }
            const double recs = (double)nblocks * BLOCK * steps;
            printf("{\"table_bytes\": %zu, \"variant\": \"%s\", \"ms\": %.4f, \"Grec_per_s\": %.2f, "
                   "\"CU_cycles_per_rec\": %.3f}\n",
                   bytes, v == 0 ? "own" : (v == 1 ? "coop" : "coopx"), best, recs / (best * 1e-3) / 1e9,
                   (best * 1e-3) * 2.4e9 * 256 / recs);
        }
        CHK(hipFree(d_tab));
    }
    return 0;
}
