// HBM copy-rate probe (tools/, not the product): 1 GiB device-to-device copies in a few
// shapes, to pick the reference rate bench.py prices fractions against (dc_copy_probe).
//   hipcc --offload-arch=gfx950 -O3 tools/copy_probe.hip -o tools/_copy_probe && tools/_copy_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(const uint4 *__restrict__ src, uint4 *__restrict__ dst, uint64_t n16)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        uint4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const uint4 *p = src + i + k * stride;
            if (NT) v[k] = make_uint4(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y),
                                      __builtin_nontemporal_load(&p->z), __builtin_nontemporal_load(&p->w));
            else v[k] = *p;
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            uint4 *p = dst + i + k * stride;
            if (NT) {
                __builtin_nontemporal_store(v[k].x, &p->x);
                __builtin_nontemporal_store(v[k].y, &p->y);
                __builtin_nontemporal_store(v[k].z, &p->z);
                __builtin_nontemporal_store(v[k].w, &p->w);
            } else {
                *p = v[k];
            }
        }
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}

template <int U, bool NT>
static float run(const uint4 *s, uint4 *d, uint64_t n16, int grid)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_copy<U, NT><<<grid, 256>>>(s, d, n16);
    hipEventRecord(a);
    for (int r = 0; r < 10; ++r) k_copy<U, NT><<<grid, 256>>>(s, d, n16);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 10;
}

int main()
{
    const uint64_t bytes = 1ull << 30, n16 = bytes / 16;
    uint4 *s, *d;
    if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 1;
    hipMemset(s, 1, bytes);
    hipMemset(d, 0, bytes);
    const int grids[] = {1024, 2048, 4096, 8192, 16384};
    for (int g : grids) {
        const float t[6] = {run<1, false>(s, d, n16, g), run<4, false>(s, d, n16, g), run<8, false>(s, d, n16, g),
                            run<1, true>(s, d, n16, g), run<4, true>(s, d, n16, g), run<8, true>(s, d, n16, g)};
        printf("grid %5d  GB/s (read+write):", g);
        const char *nm[6] = {"u1", "u4", "u8", "u1nt", "u4nt", "u8nt"};
        for (int k = 0; k < 6; ++k) printf(" %s %.0f", nm[k], 2.0 * bytes / (t[k] * 1e-3) / 1e9);
        printf("\n");
    }
    return 0;
}
