// Scalar MTF resolve step check (tools only): runs the SGPR-list step of k_nyb_resolve_s on a
// fixed token trace, at every start alignment, and prints the per-step byte and list read.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
typedef uint32_t u32x32 __attribute__((ext_vector_type(32)));
#define STEP_BODY(EXTRA)                                                                     \
        "s_lshl_b32 m0, %[ctx], 1\n\t"                                                      \
        "s_mul_i32 s98, %[t], 0x1010101\n\t"                                                \
        "s_mov_b32 s99, s98\n\t"                                                            \
        "s_movrels_b64 s[96:97], s[64:65]\n\t" EXTRA                                        \
        "s_xor_b64 s[98:99], s[98:99], s[96:97]\n\t"                                        \
        "s_sub_u32 s100, s98, 0x1010101\n\t"                                                \
        "s_subb_u32 s101, s99, 0x1010101\n\t"                                               \
        "s_andn2_b64 s[100:101], s[100:101], s[98:99]\n\t"                                  \
        "s_and_b64 s[100:101], s[100:101], %[h80]\n\t"                                      \
        "s_ff1_i32_b64 s98, s[100:101]\n\t"                                                 \
        "s_lshr_b32 s98, s98, 3\n\t"                                                        \
        "s_min_u32 s98, s98, 7\n\t"                                                         \
        "s_and_b32 s99, %[t], 7\n\t"                                                        \
        "s_bitcmp1_b32 %[t], 7\n\t"                                                         \
        "s_cselect_b32 s98, s99, s98\n\t"                                                   \
        "s_lshl_b32 s99, s99, 3\n\t"                                                        \
        "s_lshr_b64 s[100:101], s[96:97], s99\n\t"                                          \
        "s_and_b32 s100, s100, 0xff\n\t"                                                    \
        "s_bitcmp1_b32 %[t], 7\n\t"                                                         \
        "s_cselect_b32 %[v], s100, %[t]\n\t"                                                \
        "s_lshl_b32 s99, s98, 3\n\t"                                                        \
        "s_lshl_b64 s[100:101], %[ff00], s99\n\t"                                           \
        "s_lshl_b64 s[98:99], s[96:97], 8\n\t"                                              \
        "s_xor_b64 s[98:99], s[98:99], s[96:97]\n\t"                                        \
        "s_andn2_b64 s[98:99], s[98:99], s[100:101]\n\t"                                    \
        "s_xor_b64 s[96:97], s[96:97], s[98:99]\n\t"                                        \
        "s_or_b32 s96, s96, %[v]\n\t"                                                       \
        "s_movreld_b64 s[64:65], s[96:97]\n\t"                                              \
        "s_bfe_u32 %[ctx], %[v], 0x40003"

__global__ void k_trace(const uint8_t *tok, int n, uint32_t ctx0, uint32_t *ov, uint64_t *oL, uint32_t *octx)
{
    const uint64_t h80 = 0x8080808080808080ull, ff00 = 0xFFFFFFFFFFFFFF00ull, L0 = 0x736e696f61746520ull;
    u32x32 lists;
    for (int c = 0; c < 16; ++c) { lists[2 * c] = (uint32_t)L0; lists[2 * c + 1] = (uint32_t)(L0 >> 32); }
    uint32_t ctx = ctx0;
    const uint32_t tv = threadIdx.x < (unsigned)n ? tok[threadIdx.x] : 0u;
    for (int i = 0; i < n; ++i) {
        uint32_t v, t = (uint32_t)__builtin_amdgcn_readlane((int)tv, i);
        uint64_t Lr;
        octx[i] = ctx;
        asm volatile(STEP_BODY("s_mov_b64 %[Lr], s[96:97]\n\t")
                     : [lists] "+{s[64:95]}"(lists), [ctx] "+s"(ctx), [v] "=&s"(v), [Lr] "=&s"(Lr)
                     : [t] "s"(t), [h80] "s"(h80), [ff00] "s"(ff00)
                     : "s96", "s97", "s98", "s99", "s100", "s101", "scc");
        if (threadIdx.x == 0) { ov[i] = v; oL[i] = Lr; }
    }
}

// same, without the debug copy and with no stores inside the loop (the product's shape)
__global__ void k_plain(const uint8_t *tok, int n, uint32_t ctx0, uint8_t *out)
{
    const uint64_t h80 = 0x8080808080808080ull, ff00 = 0xFFFFFFFFFFFFFF00ull, L0 = 0x736e696f61746520ull;
    u32x32 lists;
    for (int c = 0; c < 16; ++c) { lists[2 * c] = (uint32_t)L0; lists[2 * c + 1] = (uint32_t)(L0 >> 32); }
    uint32_t ctx = ctx0, ovv = 0;
    const int lane = threadIdx.x;
    const uint32_t tv = lane < n ? tok[lane] : 0u;
    for (int i = 0; i < n; ++i) {
        uint32_t v, t = (uint32_t)__builtin_amdgcn_readlane((int)tv, i);
        asm volatile(STEP_BODY("")
                     : [lists] "+{s[64:95]}"(lists), [ctx] "+s"(ctx), [v] "=&s"(v)
                     : [t] "s"(t), [h80] "s"(h80), [ff00] "s"(ff00)
                     : "s96", "s97", "s98", "s99", "s100", "s101", "scc");
        ovv = lane == i ? v : ovv;
    }
    if (lane < n) out[lane] = (uint8_t)ovv;
}

int main()
{
    const uint8_t toks[15] = {0x83, 0x79, 0x80, 0x77, 0x82, 0x6c, 0x6c, 0x81, 0x86, 0x80, 0x80, 0x87, 0x81, 0x84, 0x68};
    const char *want = "ay well i in th";
    uint8_t *dt, *dout;
    uint32_t *dv, *dc;
    uint64_t *dL;
    hipMalloc(&dt, 64); hipMalloc(&dout, 64); hipMalloc(&dv, 64 * 4); hipMalloc(&dc, 64 * 4); hipMalloc(&dL, 64 * 8);
    hipMemcpy(dt, toks, 15, hipMemcpyHostToDevice);
    const uint32_t ctx0 = ('w' >> 3) & 15;
    k_trace<<<1, 64>>>(dt, 15, ctx0, dv, dL, dc);
    uint32_t hv[15], hc[15];
    uint64_t hL[15];
    hipMemcpy(hv, dv, 60, hipMemcpyDeviceToHost); hipMemcpy(hL, dL, 120, hipMemcpyDeviceToHost);
    hipMemcpy(hc, dc, 60, hipMemcpyDeviceToHost);
    for (int i = 0; i < 15; ++i) {
        char ls[9];
        for (int k = 0; k < 8; ++k) ls[k] = (char)(hL[i] >> (8 * k));
        ls[8] = 0;
        printf("trace step %2d tok %02x ctx %2u list '%s' -> '%c' (want '%c')\n", i + 1, toks[i], hc[i], ls, (char)hv[i], want[i]);
    }
    uint8_t ho[16] = {0};
    k_plain<<<1, 64>>>(dt, 15, ctx0, dout);
    hipMemcpy(ho, dout, 15, hipMemcpyDeviceToHost);
    printf("plain: '%.15s' %s\n", (char *)ho, memcmp(ho, want, 15) ? "FAIL" : "ok");
    return 0;
}
