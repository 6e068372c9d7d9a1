// HBM reference-rate shapes (tools only): which 1 GiB copy / read shape reaches the guide's
// ~6.3 TB/s float4 copy (MI355X_MICROARCH.md chip table) on this box. HIP-event timing, mean of
// 20 launches after a ~0.5 s clock pre-warm. Prints one line per shape: read+write TB/s.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/copy_shapes.hip -o /tmp/copy_shapes
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int U, bool NT>   // U uint4 per lane per grid step, all loads issued before the stores
__global__ __launch_bounds__(256) void k_copy(const uint4 *__restrict__ s, uint4 *__restrict__ d, uint64_t n)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n; i += stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + (uint64_t)u * 256;
            if (NT) {
                const uint32_t *q = reinterpret_cast<const uint32_t *>(s + j);
                v[u] = j < n ? make_uint4(__builtin_nontemporal_load(q), __builtin_nontemporal_load(q + 1),
                                          __builtin_nontemporal_load(q + 2), __builtin_nontemporal_load(q + 3))
                             : make_uint4(0, 0, 0, 0);
            } else {
                v[u] = j < n ? s[j] : make_uint4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + (uint64_t)u * 256;
            if (j >= n) break;
            if (NT) {
                uint32_t *w = reinterpret_cast<uint32_t *>(d + j);
                __builtin_nontemporal_store(v[u].x, w); __builtin_nontemporal_store(v[u].y, w + 1);
                __builtin_nontemporal_store(v[u].z, w + 2); __builtin_nontemporal_store(v[u].w, w + 3);
            } else {
                d[j] = v[u];
            }
        }
    }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_read(const uint4 *__restrict__ s, uint64_t n, uint32_t *out)
{
    uint32_t a = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n; i += stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + (uint64_t)u * 256;
            if (j < n) {
                const uint32_t *q = reinterpret_cast<const uint32_t *>(s + j);
                if (NT) a ^= __builtin_nontemporal_load(q) ^ __builtin_nontemporal_load(q + 1) ^
                             __builtin_nontemporal_load(q + 2) ^ __builtin_nontemporal_load(q + 3);
                else a ^= q[0] ^ q[1] ^ q[2] ^ q[3];
            }
        }
    }
    if (a == 0x12345678u) out[0] = a;
}

// LDS-DMA read stream: each wave pulls 1 KiB pieces into a private LDS ring (no consumer)
template <int DEPTH>
__global__ __launch_bounds__(256) void k_read_glds(const uint4 *__restrict__ s, uint64_t n, uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint4 ring[4][DEPTH][64];
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    int slot = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + (uint64_t)w * 64; i < n; i += stride) {
        __builtin_amdgcn_global_load_lds((const void *)(s + i + lane),
                                         (__attribute__((address_space(3))) void *)&ring[w][slot][0], 16, 0, 2);
        slot = (slot + 1) % DEPTH;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (ring[w][0][lane].x == 0x12345678u) out[0] = 1;
}

static float timeit(void (*launch)(void *), void *arg, int reps)
{
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    launch(arg);
    hipEventRecord(a);
    for (int r = 0; r < reps; ++r) launch(arg);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a); hipEventDestroy(b);
    return ms / reps;
}

struct Arg { const uint4 *s; uint4 *d; uint64_t n; uint32_t *o; int grid; };
#define COPY(U, NT) [](void *p) { Arg *q = (Arg *)p; k_copy<U, NT><<<q->grid, 256>>>(q->s, q->d, q->n); }
#define READ(U, NT) [](void *p) { Arg *q = (Arg *)p; k_read<U, NT><<<q->grid, 256>>>(q->s, q->n, q->o); }
#define GLDS(D) [](void *p) { Arg *q = (Arg *)p; k_read_glds<D><<<q->grid, 256>>>(q->s, q->n, q->o); }

int main()
{
    const uint64_t bytes = 1ull << 30, n = bytes / 16;
    uint4 *s, *d; uint32_t *o;
    if (hipMalloc(&s, bytes) || hipMalloc(&d, bytes) || hipMalloc(&o, 64)) { printf("alloc failed\n"); return 1; }
    hipMemset(s, 1, bytes);
    hipDeviceSynchronize();
    Arg A{s, d, n, o, 16384};
    for (int r = 0; r < 300; ++r) k_copy<1, true><<<16384, 256>>>(s, d, n);   // clock pre-warm
    hipDeviceSynchronize();
    const int grids[] = {1024, 2048, 4096, 8192, 16384, 32768, 65536, 262144};
    struct V { const char *name; void (*f)(void *); int U; bool copy; } vs[] = {
        {"copy U1 nt", COPY(1, true), 1, true},   {"copy U1 plain", COPY(1, false), 1, true},
        {"copy U2 nt", COPY(2, true), 2, true},   {"copy U4 nt", COPY(4, true), 4, true},
        {"copy U4 plain", COPY(4, false), 4, true}, {"copy U8 nt", COPY(8, true), 8, true},
        {"read U1 nt", READ(1, true), 1, false},  {"read U4 nt", READ(4, true), 4, false},
        {"read U4 plain", READ(4, false), 4, false}, {"read glds d4", GLDS(4), 1, false},
        {"read glds d8", GLDS(8), 1, false},
    };
    for (auto &v : vs) {
        for (int g : grids) {
            if ((uint64_t)g * 256 * v.U > n) continue;
            A.grid = g;
            const float ms = timeit(v.f, &A, 20);
            const double tbs = (v.copy ? 2.0 : 1.0) * bytes / (ms * 1e-3) / 1e12;
            printf("%-16s grid %6d  %.4f ms  %.3f TB/s\n", v.name, g, ms, tbs);
        }
    }
    return 0;
}
