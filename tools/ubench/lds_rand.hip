// Micro-benchmark: dependent chains of random 16-bit LDS lookups (the Huffman decoder's
// inner pattern: x -> lut[x & 4095] -> shift -> next). Reports lookups per CU-cycle for
// several (waves per workgroup, chains per lane). One workgroup per CU, 256 workgroups.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int NC>
__global__ void k_chain(const uint16_t *__restrict__ glut, uint32_t iters, uint32_t *__restrict__ out)
{
    __shared__ uint16_t lut[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) lut[i] = glut[i];
    __syncthreads();
    uint32_t x[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) x[j] = (threadIdx.x * 2654435761u) ^ (j * 40503u) ^ (blockIdx.x * 97u);
    for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const uint32_t e = lut[x[j] & 4095u];
            x[j] = (x[j] >> (e & 7u)) ^ (e * 2654435761u);
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < NC; ++j) s ^= x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NC>
static void run(int nw, const uint16_t *d_lut, uint32_t *d_out)
{
    const uint32_t iters = 4096;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k_chain<NC><<<256, nw * 64>>>(d_lut, iters, d_out);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) k_chain<NC><<<256, nw * 64>>>(d_lut, iters, d_out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    const double wave_lookups = (double)nw * NC * iters;   // per CU, wave instructions
    const double cyc = ms * 1e-3 * 2.4e9;
    printf("waves %2d chains %d : %.3f ms  %.1f CU-cycles per wave-lookup  (%.2f lane-lookups/ns chip)\n", nw, NC, ms,
           cyc / wave_lookups, 256.0 * wave_lookups * 64 / (ms * 1e6));
}

int main()
{
    uint16_t h[4096];
    uint32_t s = 12345;
    for (int i = 0; i < 4096; ++i) { s = s * 1103515245u + 12345u; h[i] = (uint16_t)(s >> 16); }
    uint16_t *d_lut; uint32_t *d_out;
    hipMalloc(&d_lut, sizeof(h)); hipMalloc(&d_out, 256 * 1024 * 4);
    hipMemcpy(d_lut, h, sizeof(h), hipMemcpyHostToDevice);
    for (int nw : {4, 8, 16}) { run<1>(nw, d_lut, d_out); run<2>(nw, d_lut, d_out); run<4>(nw, d_lut, d_out); run<8>(nw, d_lut, d_out); }
    return 0;
}
