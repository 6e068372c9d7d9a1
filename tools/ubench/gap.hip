// Inter-kernel gap probe (tools only): K dependent launches on one stream, as plain launches
// and as one captured hipGraph, for an empty kernel and a 64 MiB copy.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
__global__ void k_empty(int *p) { if (p && threadIdx.x == 1024) *p = 0; }
__global__ __launch_bounds__(256) void k_copy(const uint4 *s, uint4 *d, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) d[i] = s[i];
}
static float timeit(hipStream_t st, void (*body)(hipStream_t, void *), void *a, int reps)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    body(st, a);
    hipEventRecord(e0, st);
    for (int r = 0; r < reps; ++r) body(st, a);
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}
struct A { uint4 *s, *d; uint64_t n; int k; int grid; hipGraphExec_t g; };
static void plain_empty(hipStream_t st, void *p) { A *a = (A *)p; for (int i = 0; i < a->k; ++i) k_empty<<<a->grid, 256, 0, st>>>(nullptr); }
static void plain_copy(hipStream_t st, void *p) { A *a = (A *)p; for (int i = 0; i < a->k; ++i) k_copy<<<a->grid, 256, 0, st>>>(a->s, a->d, a->n); }
static void graph(hipStream_t st, void *p) { A *a = (A *)p; hipGraphLaunch(a->g, st); }
int main()
{
    hipStream_t st; hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    A a; a.n = (64ull << 20) / 16; hipMalloc(&a.s, 64 << 20); hipMalloc(&a.d, 64 << 20); a.k = 20;
    for (int grid : {1, 1024, 16384}) {
        a.grid = grid;
        float pe = timeit(st, plain_empty, &a, 20);
        hipGraph_t g; hipStreamBeginCapture(st, hipStreamCaptureModeGlobal); plain_empty(st, &a); hipStreamEndCapture(st, &g);
        hipGraphInstantiate(&a.g, g, nullptr, nullptr, 0);
        float ge = timeit(st, graph, &a, 20);
        printf("empty grid %5d: plain %.2f us/launch, graph %.2f us/launch\n", grid, pe * 1000 / a.k, ge * 1000 / a.k);
        hipGraphExecDestroy(a.g); hipGraphDestroy(g);
    }
    a.grid = 4096;
    float pc = timeit(st, plain_copy, &a, 10);
    hipGraph_t g; hipStreamBeginCapture(st, hipStreamCaptureModeGlobal); plain_copy(st, &a); hipStreamEndCapture(st, &g);
    hipGraphInstantiate(&a.g, g, nullptr, nullptr, 0);
    float gc = timeit(st, graph, &a, 10);
    printf("64 MiB copy: plain %.2f us/launch, graph %.2f us/launch\n", pc * 1000 / a.k, gc * 1000 / a.k);
    return 0;
}
