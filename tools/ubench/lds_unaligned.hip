// Does ds_write_b32 / ds_read_b32 at a byte (unaligned) LDS address work on this box, and
// what does it cost? Writes 4 bytes at offsets 0..7 and reads the LDS back bytewise; then
// times 4096 unaligned vs aligned stores per lane.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void k_check(uint8_t *out)
{
    __shared__ uint32_t s[64];
    const int t = threadIdx.x;
    if (t < 64) s[t] = 0;
    __syncthreads();
    if (t < 8) {
        uint32_t addr = (uint32_t)(uintptr_t)(reinterpret_cast<uint8_t *>(s) + 8 * t + (t & 3));
        uint32_t v = 0x44332211u + 0x01010101u * t;
        asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(v) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        uint32_t r;
        asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr) : "memory");
        reinterpret_cast<uint32_t *>(out + 256)[t] = r;
    }
    __syncthreads();
    if (t < 64) reinterpret_cast<uint32_t *>(out)[t] = s[t];
}

template <int UNAL>
__global__ void k_time(uint32_t *sink, int iters)
{
    __shared__ uint8_t s[64 * 72 + 64];
    const int lane = threadIdx.x & 63;
    uint32_t base = (uint32_t)(uintptr_t)(s + (threadIdx.x >> 6) * 0) + lane * 68;
    uint32_t acc = lane;
    for (int i = 0; i < iters; ++i) {
        uint32_t a = base + (UNAL ? ((i * 3 + lane) & 63) : ((i * 4) & 60));
        asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(acc) : "memory");
        acc += 7;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (acc == 12345) sink[0] = acc;
}

int main()
{
    uint8_t *d, h[512];
    hipMalloc(&d, 512);
    hipMemset(d, 0, 512);
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    for (int t = 0; t < 8; ++t) {
        printf("t=%d off=%d: ", t, 8 * t + (t & 3));
        for (int k = 0; k < 8; ++k) printf("%02x ", h[8 * t + k]);
        printf(" read back %08x\n", ((uint32_t *)(h + 256))[t]);
    }
    uint32_t *sink;
    hipMalloc(&sink, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
        float ms[2];
        for (int u = 0; u < 2; ++u) {
            hipEventRecord(e0);
            if (u) hipLaunchKernelGGL(k_time<1>, dim3(1024), dim3(512), 0, 0, sink, 4096);
            else hipLaunchKernelGGL(k_time<0>, dim3(1024), dim3(512), 0, 0, sink, 4096);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms[u], e0, e1);
        }
        printf("aligned %.3f ms, unaligned %.3f ms\n", ms[0], ms[1]);
    }
    return 0;
}
