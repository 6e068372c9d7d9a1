// Micro-benchmark: LDS cost of the decoder's table lookups, by table layout, on the index
// distribution of a real n=2 stream (12-bit windows at symbol starts of C2 enwik-like
// text, tools/ubench/windows.bin from gen_windows.py). Independent lookups (throughput),
// 16 waves per CU, one workgroup per CU, 256 workgroups. Prints LDS cycles per wave-lookup.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <vector>

template <int MODE>
__global__ __launch_bounds__(1024) void k_lut(const uint16_t *__restrict__ win, uint32_t nwin, uint32_t iters,
                                              uint32_t *__restrict__ out)
{
    __shared__ __attribute__((aligned(16))) uint32_t tab[16384];   // 64 KiB
    for (int i = threadIdx.x; i < 16384; i += blockDim.x) tab[i] = i * 2654435761u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    uint32_t w[16];
    const uint32_t base = ((blockIdx.x * 1024u + threadIdx.x) * 16u * 7u) % (nwin - 16);
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = win[base + j];
    // precomputed byte addresses (VALU cost not measured)
    uint32_t a[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t x = w[j];
        if (MODE == 0) a[j] = (x & 4095u) * 2u;                 // u16, 4096 entries (8 KiB)
        if (MODE == 1) a[j] = (x & 63u) * 2u;                   // u16, 64 entries
        if (MODE == 2) a[j] = (x & 127u) * 2u;                  // u16, 128 entries
        if (MODE == 3) a[j] = (x & 255u) * 2u;                  // u16, 256 entries
        if (MODE == 4) a[j] = ((x & 511u) << 7) | ((lane & 31) << 2);   // lane-banked dwords, 512 entries
        if (MODE == 5) a[j] = (x & 4095u) * 8u;                 // u64, 4096 entries (32 KiB)
        if (MODE == 6) a[j] = (x & 4095u) * 4u;                 // u32, 4096 entries (16 KiB)
        if (MODE == 7) a[j] = (x & 1023u) * 2u;                 // u16, 1024 entries
        if (MODE == 8) a[j] = (__builtin_bitreverse32(x) >> 20) * 2u;   // u16 x4096, MSB-first index
        if (MODE == 9) a[j] = ((lane * 69u + j * 7u) % 2100u) * 4u;       // stage-window dword reads
    }
    uint32_t s = 0;
    const char *tb = reinterpret_cast<const char *>(tab);
    for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (MODE == 5) {
                const uint2 v = *reinterpret_cast<const uint2 *>(tb + a[j]);
                s += v.x ^ v.y;
            } else if (MODE == 9) {
                const uint32_t *p = reinterpret_cast<const uint32_t *>(tb + a[j]);
                s += p[0] ^ p[1] ^ p[2];
            } else if (MODE == 4 || MODE == 6) {
                s += *reinterpret_cast<const uint32_t *>(tb + a[j]);
            } else {
                s += *reinterpret_cast<const uint16_t *>(tb + a[j]);
            }
        }
        asm volatile("" : "+v"(s));
    }
    out[blockIdx.x * 1024 + threadIdx.x] = s;
}

template <int MODE>
static void run(const char *name, const uint16_t *d_win, uint32_t nwin, uint32_t *d_out)
{
    const uint32_t iters = 2048;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k_lut<MODE><<<256, 1024>>>(d_win, nwin, iters, d_out);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) k_lut<MODE><<<256, 1024>>>(d_win, nwin, iters, d_out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    const double wave_lookups = 16.0 * 16 * iters;   // per CU
    printf("mode %d %-34s %.3f ms  %.2f CU-cycles per wave-lookup (2.4 GHz)\n", MODE, name, ms,
           ms * 1e-3 * 2.4e9 / wave_lookups);
}

int main(int argc, char **argv)
{
    const char *path = argc > 1 ? argv[1] : "tools/ubench/windows.bin";
    FILE *f = fopen(path, "rb");
    if (!f) { printf("no %s\n", path); return 1; }
    std::vector<uint16_t> w(1 << 22);
    const size_t nw = fread(w.data(), 2, w.size(), f);
    fclose(f);
    uint16_t *d_win; uint32_t *d_out;
    hipMalloc(&d_win, nw * 2); hipMalloc(&d_out, 256 * 1024 * 4);
    hipMemcpy(d_win, w.data(), nw * 2, hipMemcpyHostToDevice);
    run<0>("u16 x4096 (current 12-bit LUT)", d_win, nw, d_out);
    run<1>("u16 x64 (6-bit)", d_win, nw, d_out);
    run<2>("u16 x128 (7-bit)", d_win, nw, d_out);
    run<3>("u16 x256 (8-bit)", d_win, nw, d_out);
    run<7>("u16 x1024 (10-bit)", d_win, nw, d_out);
    run<4>("lane-banked u32 x512 (9-bit)", d_win, nw, d_out);
    run<6>("u32 x4096", d_win, nw, d_out);
    run<5>("u64 x4096 (ds_read_b64)", d_win, nw, d_out);
    run<8>("u16 x4096 MSB-first index", d_win, nw, d_out);
    run<9>("3 stage dwords (per 3 reads)", d_win, nw, d_out);
    // uniform random indices for comparison
    for (size_t i = 0; i < nw; ++i) w[i] = (uint16_t)((i * 2654435761u) >> 7);
    hipMemcpy(d_win, w.data(), nw * 2, hipMemcpyHostToDevice);
    printf("-- uniform random indices --\n");
    run<0>("u16 x4096", d_win, nw, d_out);
    run<6>("u32 x4096", d_win, nw, d_out);
    run<5>("u64 x4096", d_win, nw, d_out);
    return 0;
}
