// Micro-benchmark of the S=64 decoder's batch (tools/ubench): NC chains per lane decode
// 4 symbols per batch from an LDS stage through a 16-bit LUT, variants isolating parts.
//   V=0 full batch (3-word window reads + 4 lookups, 64-bit shifts)
//   V=1 window kept in registers (no stage reads; window += lookups)
//   V=2 full batch, 32-bit alignbit extraction instead of v_lshrrev_b64
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int NC, int V>
__global__ void k_dec(const uint16_t *__restrict__ glut, const uint32_t *__restrict__ gstage, uint32_t batches,
                      uint32_t *__restrict__ out)
{
    __shared__ uint16_t lut[4096];
    __shared__ uint32_t stage[32][1088];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) lut[i] = glut[i];
    for (int i = threadIdx.x; i < 32 * 1088; i += blockDim.x) (&stage[0][0])[i] = gstage[i & 4095];
    __syncthreads();
    const uint32_t *st[NC];
    uint32_t c[NC], acc[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) { st[j] = stage[(w * NC + j) & 31]; c[j] = lane * 35 * 8; acc[j] = 0; }
    uint64_t wreg[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) wreg[j] = ((uint64_t)gstage[lane] << 32) | gstage[lane + 7];
    for (uint32_t b = 0; b < batches; ++b) {
        uint64_t win[NC];
        uint32_t off[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            if (V == 1) {
                win[j] = wreg[j];
            } else {
                const uint32_t a = (c[j] >> 5) & 1023;
                const uint32_t w0 = st[j][a], w1 = st[j][a + 1], w2 = st[j][a + 2];
                win[j] = ((uint64_t)__builtin_amdgcn_alignbit(w2, w1, c[j]) << 32) | __builtin_amdgcn_alignbit(w1, w0, c[j]);
            }
            off[j] = 0;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t e[NC], mn = 255;
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                uint32_t x;
                if (V == 2) x = __builtin_amdgcn_alignbit((uint32_t)(win[j] >> 32), (uint32_t)win[j], off[j]);
                else x = (uint32_t)(win[j] >> off[j]);
                e[j] = lut[x & 4095u];
            }
#pragma unroll
            for (int j = 0; j < NC; ++j) mn = min(mn, e[j] & 255u);
            if (__builtin_expect(__any(mn == 0), 0)) {
#pragma unroll
                for (int j = 0; j < NC; ++j) e[j] |= 1;
            }
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                acc[j] = __builtin_amdgcn_perm(e[j], acc[j], 0x05020100u);
                off[j] += e[j] & 255u;
            }
        }
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            c[j] += off[j];
            if (V == 1) wreg[j] = (wreg[j] >> 7) ^ ((uint64_t)off[j] << 40);
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < NC; ++j) s ^= acc[j] ^ c[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NC, int V>
static void run(int nw, const uint16_t *d_lut, const uint32_t *d_stage, uint32_t *d_out)
{
    const uint32_t batches = 1024;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k_dec<NC, V><<<256, nw * 64>>>(d_lut, d_stage, batches, d_out);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) k_dec<NC, V><<<256, nw * 64>>>(d_lut, d_stage, batches, d_out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    const double wave_syms = (double)nw * NC * batches * 4;   // per CU
    printf("V%d waves %2d chains %d : %.3f ms  %.1f CU-cycles per wave-symbol\n", V, nw, NC, ms,
           ms * 1e-3 * 2.4e9 / wave_syms);
}

int main()
{
    static uint16_t h[4096];
    static uint32_t hs[4096];
    uint32_t s = 12345;
    for (int i = 0; i < 4096; ++i) {   // lengths 2..9 (never 0), symbol byte random
        s = s * 1103515245u + 12345u;
        h[i] = (uint16_t)(2 + ((s >> 16) % 8)) | (uint16_t)(((s >> 8) & 255) << 8);
        hs[i] = s ^ (s >> 13);
    }
    uint16_t *d_lut; uint32_t *d_out, *d_stage;
    hipMalloc(&d_lut, sizeof(h)); hipMalloc(&d_out, 256 * 1024 * 4); hipMalloc(&d_stage, sizeof(hs));
    hipMemcpy(d_lut, h, sizeof(h), hipMemcpyHostToDevice);
    hipMemcpy(d_stage, hs, sizeof(hs), hipMemcpyHostToDevice);
    run<2, 0>(16, d_lut, d_stage, d_out);
    run<2, 1>(16, d_lut, d_stage, d_out);
    run<2, 2>(16, d_lut, d_stage, d_out);
    run<4, 0>(8, d_lut, d_stage, d_out);
    run<1, 0>(16, d_lut, d_stage, d_out);
    run<2, 0>(8, d_lut, d_stage, d_out);
    return 0;
}
