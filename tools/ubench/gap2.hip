// What sets the gap between dependent kernels (tools only; run under rocprofv3 --kernel-trace):
// 10 back-to-back launches each of an empty grid, a 1 GiB read-only sum, a 1 GiB copy with
// default stores and one with streaming (nt) stores.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
__global__ __launch_bounds__(256) void k_empty(int *p) { if (p && threadIdx.x == 1024) *p = 0; }
__global__ __launch_bounds__(256) void k_sum(const uint4 *s, uint64_t n, uint32_t *out)
{
    uint32_t a = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t *q = reinterpret_cast<const uint32_t *>(s + i);
        a ^= __builtin_nontemporal_load(q) ^ __builtin_nontemporal_load(q + 1) ^ __builtin_nontemporal_load(q + 2) ^
             __builtin_nontemporal_load(q + 3);
    }
    if (a == 0x12345678u) out[0] = a;
}
template <bool NT>
__global__ __launch_bounds__(256) void k_copy(const uint4 *s, uint4 *d, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t *q = reinterpret_cast<const uint32_t *>(s + i);
        uint32_t *w = reinterpret_cast<uint32_t *>(d + i);
        const uint32_t a = __builtin_nontemporal_load(q), b = __builtin_nontemporal_load(q + 1),
                       c = __builtin_nontemporal_load(q + 2), e = __builtin_nontemporal_load(q + 3);
        if (NT) {
            __builtin_nontemporal_store(a, w); __builtin_nontemporal_store(b, w + 1);
            __builtin_nontemporal_store(c, w + 2); __builtin_nontemporal_store(e, w + 3);
        } else {
            d[i] = make_uint4(a, b, c, e);
        }
    }
}
int main()
{
    const uint64_t bytes = 1ull << 30, n = bytes / 16;
    uint4 *s, *d; uint32_t *o;
    hipMalloc(&s, bytes); hipMalloc(&d, bytes); hipMalloc(&o, 64);
    hipMemset(s, 1, bytes);
    hipDeviceSynchronize();
    for (int r = 0; r < 10; ++r) k_empty<<<16384, 256>>>(nullptr);
    hipDeviceSynchronize();
    for (int r = 0; r < 10; ++r) k_sum<<<16384, 256>>>(s, n, o);
    hipDeviceSynchronize();
    for (int r = 0; r < 10; ++r) k_copy<false><<<16384, 256>>>(s, d, n);
    hipDeviceSynchronize();
    for (int r = 0; r < 10; ++r) k_copy<true><<<16384, 256>>>(s, d, n);
    hipDeviceSynchronize();
    for (int r = 0; r < 10; ++r) { k_copy<true><<<16384, 256>>>(s, d, n); k_sum<<<16384, 256>>>(d, n, o); }
    hipDeviceSynchronize();
    printf("done\n");
    return 0;
}
