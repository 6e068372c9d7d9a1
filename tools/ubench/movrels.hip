// s_movrels_b64 / s_movreld_b64: is M0 counted in dwords or in 64-bit registers? (tools only)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t u32x32 __attribute__((ext_vector_type(32)));
__global__ void k(uint32_t *out, uint32_t m0)
{
    u32x32 r;
    for (int i = 0; i < 32; ++i) r[i] = 100 + i;
    uint32_t lo, hi;
    uint64_t w = 0xAAAABBBBCCCCDDDDull;
    asm volatile("s_mov_b32 m0, %[m]\n\ts_nop 1\n\ts_movrels_b64 s[96:97], s[64:65]\n\ts_mov_b32 %[lo], s96\n\ts_mov_b32 %[hi], s97\n\t"
                 "s_movreld_b64 s[64:65], %[w]"
                 : [r] "+{s[64:95]}"(r), [lo] "=&s"(lo), [hi] "=&s"(hi) : [m] "s"(m0), [w] "s"(w) : "s96", "s97");
    if (threadIdx.x == 0) {
        out[0] = lo; out[1] = hi;
        for (int i = 0; i < 32; ++i) out[2 + i] = r[i];
    }
}
int main()
{
    uint32_t *d, h[34];
    hipMalloc(&d, sizeof(h));
    for (uint32_t m = 0; m < 4; ++m) {
        k<<<1, 64>>>(d, m);
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        printf("M0=%u read (%u, %u); written at:", m, h[0], h[1]);
        for (int i = 0; i < 32; ++i) if (h[2 + i] != 100u + i) printf(" s%d=%08x", 64 + i, h[2 + i]);
        printf("\n");
    }
    return 0;
}
