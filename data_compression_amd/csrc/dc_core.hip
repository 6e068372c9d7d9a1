// dc_core.hip -- gfx950 (MI355X) kernels + the device-resident extended C-ABI (dc_gpu.h).
//
// Hot path: byte histogram (H1) -> n-ary Huffman lengths (H2-H5) ->
// canonical n-ary codes (H6) -> bit packing (H7) -> decode (H8); nybble codec (N1-N7);
// small front-end (small_compression.c:507-665). Everything here is integer/byte work
// and HBM-bound: no MFMA. Design notes and the roofline per kernel: DESIGN.md.
//
// Built by data_compression_amd/build.py:
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared -> data_compression_amd/lib/libdc_core.so

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

#include <atomic>
#include <type_traits>

#include "dc_gpu.h"

#define DC_VERSION "dc-mi355x 0.1 (gfx950)"
#define DC_SYNC_GROUP 64
#define DC_SYNC_GROUP_LOG 6

// ------------------------------------------------------------------------------------
// small device helpers
// ------------------------------------------------------------------------------------
static __device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }
// a 16-B load with the streaming (nt) hint
static __device__ __forceinline__ uint4 ld_nt(const uint4 *p)
{
    return make_uint4(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y),
                      __builtin_nontemporal_load(&p->z), __builtin_nontemporal_load(&p->w));
}
// Every byte the hot kernels stream from HBM is read once per kernel, and the data they write
// is read by a later kernel only after far more than the caches hold: nt loads and stores for
// them (same-box A/B on the 1 GiB C2 step against plain ones: histogram 0.207 -> 0.188 ms,
// pack 0.379 -> 0.364, decode 0.422 -> 0.418 from the loads; the stores: see d8_out, k_huff_pack)
static __device__ __forceinline__ void st_nt(uint4 *p, const uint4 &v)
{
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
    __builtin_nontemporal_store(v.z, &p->z);
    __builtin_nontemporal_store(v.w, &p->w);
}
#define LD_HIST(p) ld_nt(p)
#define LD_PACK(p) ld_nt(p)
#define LD_DEC(p) ld_nt(p)

// 256-thread exclusive scan (u32). `scratch` holds >= 4 u32. Returns the prefix and
// the total through *total. Contains two __syncthreads().
static __device__ __forceinline__ uint32_t wg_scan_excl_u32(uint32_t v, uint32_t *scratch,
                                                            uint32_t *total)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) scratch[wid] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        uint32_t s = scratch[w];
        base += (w < wid) ? s : 0u;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// inclusive wave64 prefix sum in DPP (VALU only: __shfl_up is ds_bpermute, i.e. an LDS
// instruction queued behind the table reads): row_shr 1/2/4/8 within each row of
// 16 lanes, then row_bcast:15 and row_bcast:31 across rows (GFX9 DPP)
static __device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x)
{
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);   // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return x;
}

// SWAR byte tests on a dword (bit 7 of each byte = the test; the kernels are VALU-issue
// bound, and one 32-bit op here tests 4 bytes: 31 VALU per byte per element rule before)
static __device__ __forceinline__ uint32_t swar_eq(uint32_t x, uint32_t c4)   // byte == c
{
    const uint32_t v = x ^ c4;
    return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v) & 0x80808080u;
}
static __device__ __forceinline__ uint32_t swar_lower(uint32_t x)   // 'a' <= byte <= 'z'
{
    const uint32_t t = x & 0x7F7F7F7Fu;
    return (t + 0x1F1F1F1Fu) & ~(t + 0x05050505u) & ~x & 0x80808080u;
}

// ------------------------------------------------------------------------------------
// C5 front-end fusion (small_compression.c:582-665, then n-ary Huffman of its output M).
// M = [8, x[0]] then, for g >= 1, x[g], except that ' ' + lowercase letter at g, g + 1 (a pair
// START at g, g <= n - 2) becomes the one byte 0x80 + letter. Pairs never overlap (the second
// byte is a letter, never ' '), so the symbol stream is a per-position map of the input with
// one byte of context each side. The fused kernels read the input x itself and never write
// M: a pair's symbol is counted and coded at its SECOND position (as x[g] | 0x80: the letter
// is < 0x80) and the start position carries no symbol (in the pack: a byte value z with no
// code, 0 bits). The M order is unchanged: nothing lies between a pair's two positions.
// ------------------------------------------------------------------------------------
// The shifts must run with every lane active: a DPP read of a lane that EXEC disables returns
// 0. `lane == 0 ? a : dpp_wave_shr1(x)` is lowered as a branch (the call has a side effect),
// which ran the DPP with lane 0 off, so lane 1 read 0: call them as statements of their own
// (the opaque asm then keeps them from being sunk into a branch).
static __device__ __forceinline__ uint32_t dpp_wave_shr1(uint32_t x)   // lane l <- lane l - 1 (lane 0: 0)
{
    uint32_t r = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, false);
    asm volatile("" : "+v"(r));
    return r;
}
static __device__ __forceinline__ uint32_t dpp_wave_shl1(uint32_t x)   // lane l <- lane l + 1 (lane 63: 0)
{
    uint32_t r = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xf, 0xf, false);
    asm volatile("" : "+v"(r));
    return r;
}
// The dword a lane of the fused kernels loads beside its 16 bytes at p: lane 0 the one
// holding x[p - 1], lane 63 the one at p + 16 (the lanes between take the byte from their
// neighbours by DPP wave shifts); the others all read the wave's first dword (one address: one
// request; one unconditional load keeps the compiler's load waits counted). (r4: each re-read
// its own first dword, 64 lines per wave-instruction, and behind the nt granule loads every one
// went back to HBM: the fused histogram fetched 1.58 GB per GiB, profiles/r5z_C5_pmc_traffic.json)
static __device__ __forceinline__ uint64_t fe_edge_addr(uint64_t p, int lane, uint64_t n)
{
    return lane == 0 ? (p >= 4 ? p - 4 : p) : lane == 63 ? (p + 16 < n ? p + 16 : p) : p - 16 * (uint64_t)lane;
}
// pair starts among the 16 bytes w4 (q = the byte after them, 0 past the input): 0x80 in
// byte j of st[k] = a START at byte 4k + j
static __device__ __forceinline__ void fe_pair_starts(const uint32_t (&w4)[4], uint32_t q, uint32_t (&st)[4])
{
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t nx = __builtin_amdgcn_alignbyte(k < 3 ? w4[k + 1] : q, w4[k], 1u);   // the next bytes
        st[k] = swar_eq(w4[k], 0x20202020u) & swar_lower(nx);
    }
}
// a start at p - 1 (its byte pb, x[p] = the low byte of w0), which makes x[p] a pair's second
static __device__ __forceinline__ uint32_t fe_start_before(uint32_t pb, uint32_t w0, uint64_t p)
{
    const uint32_t x = w0 & 255u;
    return (p >= 16 && pb == 0x20u && x >= 'a' && x <= 'z') ? 0x80u : 0u;
}

// ------------------------------------------------------------------------------------
// (H1) byte histogram per 32 KiB block.  n_ary_huffman.c:461-493
// LDS layout: dword (bin*64 + lane) holds four 8-bit counters, one per wave of the
// workgroup. Every lane owns its own dword column, so one ds_add_u32 per input byte is
// bank-conflict free (bank = lane mod 32) whatever the byte distribution, and skewed
// text (' ' and 'e' in most lanes) does not serialise. A lane sees 128 bytes per block,
// so an 8-bit counter cannot overflow. Reduction reads and clears with a rotated column
// index so it is conflict free as well.
// ------------------------------------------------------------------------------------
struct TblLds;
static __device__ void huff_table_body(TblLds &S, const uint64_t *__restrict__ freq, int freq_is_hist256,
                                       const int32_t *__restrict__ lens_in, int M, int nary,
                                       dc_dtable *__restrict__ T, dc_tree *__restrict__ tree,
                                       const uint64_t *plan_hist, uint64_t *__restrict__ d_total,
                                       int *__restrict__ perr, int *__restrict__ perr_next);

// The table build of a fused launch (HistFuse.T set): the last workgroup out, which holds the
// final histogram, builds the code table and the encode plan total right away (no table
// launch, no plan launch: dc_huff_encode_plan)
struct HistFuse {
    dc_dtable *T;          // nullptr: histogram only
    int M, nary;
    uint64_t *d_total;     // payload bits of this input under the new code
    int *perr, *perr_next; // plan error slot of this call, and the next one (cleared)
};

// PF: full blocks whose loads are in flight ahead of the one being counted. FE (the C5 fused
// front-end): the histogram is that of the front-end output M, per 32 KiB block of the INPUT:
// a pair's symbol 0x80 + letter counts at its second position (letter | 0x80), each block's
// ' ' count loses its pair starts, and block 0 gains the type byte 8 (M[0]).
// FE shard context (dist.ShardedSmall's fused encode at world > 1: FeShard[4] int64 on the
// device, nullptr for a whole stream): the shard's global bit offset and first symbol index,
// and the input bytes either side of it, -1 past the stream's ends. A shard whose left byte is
// -1 starts the stream (the type byte 8, raw x[0]); any other has no header, its x[0] may be a
// pair's second (after the left byte) or start, and its last byte may start a pair with the
// right byte.
struct FeCtx {
    bool first;
    uint32_t lb, rb;   // the bytes either side (0 past the stream's ends: never ' ', never a letter)
};
static __device__ __forceinline__ FeCtx fe_ctx(const int64_t *shard)
{
    FeCtx f{true, 0u, 0u};
    if (shard) {
        const int64_t l = shard[2], r = shard[3];
        f.first = l < 0;
        f.lb = l < 0 ? 0u : (uint32_t)l & 255u;
        f.rb = r < 0 ? 0u : (uint32_t)r & 255u;
    }
    return f;
}

template <int PF, bool FE = false>
__global__ __launch_bounds__(256) void k_hist_blocks(const uint8_t *__restrict__ in, uint64_t n,
                                                     uint64_t nblocks, uint16_t *__restrict__ bh,
                                                     uint64_t *__restrict__ hist, uint64_t *__restrict__ hacc,
                                                     uint32_t *__restrict__ hdone, uint64_t *__restrict__ hloc,
                                                     HistFuse fuse, const int64_t *__restrict__ shard = nullptr)
{
    const FeCtx fc = fe_ctx(FE ? shard : nullptr);
    __shared__ __attribute__((aligned(16))) uint32_t cnt[256 * 64];
    __shared__ uint32_t s_last;
    __shared__ uint32_t s_ps[4];
    __shared__ uint64_t s_h[256];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t inc = 1u << (8 * wv);
    const uint32_t lane4 = 4u * (uint32_t)lane;
    char *const cbase = reinterpret_cast<char *>(cnt);
    for (int i = t; i < 256 * 16; i += 256) reinterpret_cast<uint4 *>(cnt)[i] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    const uint64_t nfull = n / DC_BLOCK_BYTES;   // blocks read as 8 x 16 B per thread
    uint64_t total = 0;                           // bin t over this workgroup's blocks (u64: any grid)
    uint32_t prevc[64];                           // bin t's 64 counter dwords after the last block
#pragma unroll
    for (int q = 0; q < 64; ++q) prevc[q] = 0u;
    // software pipeline: the next PF full blocks' loads are in flight while this block counts
    // (the LDS counters allow 2 workgroups per CU, so registers up to 256 cost no occupancy)
    uint4 v[PF][8];
    uint32_t ve[FE ? PF : 1][8];   // FE: the dwords beside each 16 B (fe_edge_addr)
    uint64_t b = blockIdx.x;
    auto issue = [&](int f, uint64_t bf) {
        const uint4 *p = reinterpret_cast<const uint4 *>(in + bf * (uint64_t)DC_BLOCK_BYTES) + t;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[f][k] = LD_HIST(p + k * 256);
        if (FE) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint64_t q = bf * (uint64_t)DC_BLOCK_BYTES + (uint64_t)k * 4096 + (uint64_t)t * 16;
                ve[FE ? f : 0][k] = *reinterpret_cast<const uint32_t *>(in + fe_edge_addr(q, lane, n));
            }
        }
    };
#pragma unroll
    for (int f = 0; f < PF; ++f) {
        const uint64_t bf = b + (uint64_t)f * gridDim.x;
        if (bf < nfull) issue(f, bf);
    }
    for (; b < nblocks; b += gridDim.x) {
        uint32_t pc = 0;   // FE: pair starts this thread saw in the block
        if (b < nfull) {
            uint4 cur[8];
            uint32_t ce[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) { cur[k] = v[0][k]; ce[k] = FE ? ve[0][k] : 0u; }
#pragma unroll
            for (int f = 0; f + 1 < PF; ++f)
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    v[f][k] = v[f + 1][k];
                    if (FE) ve[FE ? f : 0][k] = ve[FE ? f + 1 : 0][k];
                }
            const uint64_t nb = b + (uint64_t)PF * gridDim.x;
            if (nb < nfull) issue(PF - 1, nb);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                uint32_t w4[4] = {cur[k].x, cur[k].y, cur[k].z, cur[k].w};
                if (FE) {   // pair seconds -> letter | 0x80, found from the byte before each (SWAR)
                    const uint64_t p = b * (uint64_t)DC_BLOCK_BYTES + (uint64_t)k * 4096 + (uint64_t)t * 16;
                    // (the shift as a statement of its own: inside `?:` it ran in a branch, lane 0 off)
                    const uint32_t pd = dpp_wave_shr1(w4[3]);
                    const uint32_t pb = lane == 0 ? (p == 0 ? fc.lb : ce[k] >> 24) : pd >> 24;   // x[p - 1]
                    const uint32_t raw3 = w4[3];
                    uint32_t sc = 0;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint32_t pv = __builtin_amdgcn_alignbyte(w4[q], q ? w4[q - 1] : pb << 24, 3u);   // the bytes before
                        uint32_t sec = swar_eq(pv, 0x20202020u) & swar_lower(w4[q]);
                        if (q == 0 && p == 0 && fc.first) sec &= ~0x8080u;   // positions 0, 1: no pair starts at 0
                        w4[q] |= sec;
                        sc += (uint32_t)__popc(sec);
                        if (q == 0 && t == 0 && k == 0) sc -= sec & 0x80u ? 1u : 0u;   // (its start: the previous block's)
                    }
                    // the block's starts = its seconds, less the one on its first byte, plus a
                    // start on its last byte (its second: the next block's first byte)
                    if (t == 255 && k == 7) {
                        const uint32_t nx = p + 16 < n ? ce[k] & 255u : fc.rb;
                        sc += ((raw3 >> 24) == 0x20u && nx >= 'a' && nx <= 'z') ? 1u : 0u;
                    }
                    pc += sc;
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        // byte address bin*256 + lane*4 in one v_perm_b32: byte 0 = lane*4,
                        // byte 1 = byte q of the input word, bytes 2-3 = 0
                        const uint32_t addr = __builtin_amdgcn_perm(w4[j], lane4, 0x0c0c0000u | ((4u + q) << 8));
                        atomicAdd(reinterpret_cast<uint32_t *>(cbase + addr), inc);
                    }
                }
            }
        } else {
            const uint64_t base = b * (uint64_t)DC_BLOCK_BYTES;
            for (uint64_t i = base + t; i < n; i += 256) {
                uint32_t x = in[i];
                if (FE) {
                    const uint32_t pv = i >= 1 ? in[i - 1] : fc.lb;
                    const bool sec = (i >= 2 || !fc.first) && pv == 0x20 && x >= 'a' && x <= 'z';
                    const uint32_t nx = i + 1 < n ? in[i + 1] : fc.rb;
                    pc += ((i >= 1 || !fc.first) && x == 0x20u && nx >= 'a' && nx <= 'z') ? 1u : 0u;
                    x |= sec ? 0x80u : 0u;
                }
                atomicAdd(&cnt[x * 64 + lane], inc);
            }
        }
        if (FE) {
            const uint32_t ws = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_incl(pc), 63);
            if (lane == 0) s_ps[wv] = ws;
        }
        __syncthreads();
        // bin t: its 64 lane columns (16-B reads, rotated so a wave's reads spread over all
        // banks). The counters are never cleared: the block's counts are the difference to
        // the previous values, kept in this thread's registers; v_dot4_u32_u8 with
        // 0x01010101 adds the four wave fields. (Clearing them cost a 64 KiB LDS write per
        // 32 KiB block.)
        const uint4 *row = reinterpret_cast<const uint4 *>(&cnt[t * 64]);
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint4 d = row[(k + t) & 15];
            const uint32_t dn[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                // a dword is c0 + 256 c1 + 65536 c2 + 2^24 c3 (mod 2^32) of the four waves'
                // running counts (field carries included), and each c_f grows by <= 128 per
                // block, so the plain 32-bit difference holds the block's four counts as bytes
                const uint32_t x = dn[q], diff = x - prevc[4 * k + q];
                acc = __builtin_amdgcn_udot4(diff, 0x01010101u, acc, false);
                prevc[4 * k + q] = x;
            }
        }
        if (FE) {   // the block's pair starts carry no symbol; block 0 holds the type byte 8
            if (t == 0x20) acc -= s_ps[0] + s_ps[1] + s_ps[2] + s_ps[3];
            if (t == 8 && b == 0 && fc.first) acc += 1u;
        }
        bh[b * 256 + t] = (uint16_t)acc;
        total += acc;
        __syncthreads();
    }
    // this workgroup's bin totals into the context's accumulator (zero at every launch), and
    // the last workgroup out moves it to hist[] and zeroes it for the next launch: no memset
    // or reduce launch, and no workgroup waits on another (a workgroup-0 reset that the
    // others waited for assumed all of the grid resident, which ranks sharing a GPU broke)
    // The hand-off is the agent-scope release/acquire pair (cdna_hip_programming.md §6
    // Guideline 16, counter form): every thread's accumulator atomic drained, a barrier, ONE
    // release fence by thread 0 before the ticket, and in the last workgroup ONE acquire
    // fence before it reads the accumulator. (r2 used the drain alone: it relied on the
    // device-scope atomics being performed past the XCDs' L2s, which the memory model does
    // not promise; a __threadfence in every thread cost 2-5% of the kernel.)
    if (total) atomicAdd(reinterpret_cast<unsigned long long *>(&hacc[t]), total);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // keep: the fence's own wait may be dropped
        const bool last = __hip_atomic_fetch_add(hdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                          gridDim.x - 1;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        s_last = last;
    }
    __syncthreads();
    if (s_last) {
        const uint64_t hv = atomicExch(reinterpret_cast<unsigned long long *>(&hacc[t]), 0ull);
        hist[t] = hv;
        hloc[t] = hv;   // this context's own histogram (hist[] may be all-reduced in place later)
        if (t == 0) atomicExch(hdone, 0u);
        if (fuse.T) {   // the counters are free now: their LDS holds the table build
            s_h[t] = hv;
            __syncthreads();
            huff_table_body(*reinterpret_cast<TblLds *>(cnt), s_h, 1, nullptr, fuse.M, fuse.nary, fuse.T, nullptr,
                            s_h, fuse.d_total, fuse.perr, fuse.perr_next);
        }
    }
}

// ------------------------------------------------------------------------------------
// (H2-H6) code table: n-ary Huffman lengths + canonical n-ary codes + packed bit codes
// + decode tables. One workgroup.
//   * merge order: the reference re-sorts its active list with a stable bubble sort
//     before every merge (n_ary_huffman.c:672-731, :962-1002); that order is ascending
//     (count, node_index) with dummy leaves at max_leaf_value+1.. (count 1, :921-929)
//     and internal nodes numbered in creation order. Here: bitonic sort of the packed
//     keys (count<<11 | index) in LDS, then the two-queue merge (internal nodes are
//     created with non-decreasing counts, so a FIFO keeps them sorted).
//   * dummy count: (n-1) - ((k-1) % (n-1)), C remainder (:900-903), incl. its phantom
//     leaf for n = 2.
//   * canonical values (:1540-1568) with the reference's index-M quirks (:1336, :1421).
// ------------------------------------------------------------------------------------
#define TBL_SORT_MAX 2048
#define TBL_NODES 4096

struct TblLds {   // k_huff_table's LDS (also carved from k_hist_blocks' counters by its last workgroup)
    __attribute__((aligned(16))) uint64_t key[TBL_SORT_MAX];   // sort keys; then the per-length symbol bitmaps
    uint64_t q2[TBL_SORT_MAX];
    int16_t parent[TBL_NODES];
    int32_t len[DC_MAX_SYMS];
    __attribute__((aligned(16))) uint32_t cnt[DC_MAX_DIGITS + 2];
    uint32_t startv[DC_MAX_DIGITS + 2];
    uint32_t starti[DC_MAX_DIGITS + 2];
    uint32_t code[256];
    uint32_t nb[256];
    int k, mn, mx, maxbits, bad;
    int aff_lo;   // fixed8: the byte whose code is 0
    uint64_t red[4];
};
static_assert(sizeof(TblLds) <= 256 * 64 * sizeof(uint32_t), "k_hist_blocks' last workgroup builds the table in its counters' LDS");

// The value lane (lane ^ d) holds, d a power of two < 64, by VALU lane moves only (no LDS
// crossbar): quad_perm for 1 and 2, row shifts for 4, row_ror:8 (xor 8 in a 16-lane row), and
// the gfx950 permlane swaps for 16 and 32 (x swapped with itself: the first result holds the
// lower row / half twice, the second the upper one twice).
static __device__ __forceinline__ uint32_t lane_xor(uint32_t x, int d, int lane)
{
    switch (d) {
    case 1: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    case 2: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    case 4: {
        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x104, 0xf, 0xf, false);   // row_shl:4
        const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);   // row_shr:4
        return (lane & 4) ? dn : up;
    }
    case 8: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xf, 0xf, false);   // row_ror:8
    case 16: {
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (lane & 16) ? r[0] : r[1];
    }
    default: {
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (lane & 32) ? r[0] : r[1];
    }
    }
}

// inclusive wave64 prefix sum of u64 in DPP (wave_scan_incl's steps on both halves; a lane
// whose source is outside its row, or a row the row mask leaves out, adds 0)
static __device__ __forceinline__ uint64_t wave_scan_incl_u64(uint64_t x)
{
#define DC_SCAN64_STEP(ctrl, rm)                                                                          \
    {                                                                                                     \
        const uint32_t lo_ = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, ctrl, rm, 0xf, false);  \
        const uint32_t hi_ = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), ctrl, rm, 0xf, false); \
        x += ((uint64_t)hi_ << 32) | lo_;                                                                 \
    }
    DC_SCAN64_STEP(0x111, 0xf) DC_SCAN64_STEP(0x112, 0xf) DC_SCAN64_STEP(0x114, 0xf) DC_SCAN64_STEP(0x118, 0xf)
    DC_SCAN64_STEP(0x142, 0xa) DC_SCAN64_STEP(0x143, 0xc)
#undef DC_SCAN64_STEP
    return x;
}

// One wave sorts a bitonic sequence of 64 distinct u64 keys (one per lane) ascending in lane
// order: 6 compare-exchange stages on VALU lane moves, branch-free (the lower lane of a pair
// keeps the smaller key: it takes its partner's when that is smaller, the upper lane when it is
// larger; keys are distinct, or equal INF pads, so one compare decides both)
static __device__ __forceinline__ uint64_t wave_bitonic_merge(uint64_t k, int lane)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t plo = lane_xor((uint32_t)k, d, lane), phi = lane_xor((uint32_t)(k >> 32), d, lane);
        const uint64_t p = ((uint64_t)phi << 32) | plo;
        const bool take = (p < k) != ((lane & d) != 0);
        k = take ? p : k;
    }
    return k;
}

// (H3) the batched two-queue n-ary merge by one wave (generate_huffman_tree, n_ary_huffman.c:
// 868-1005, whose stable re-sort :672-731 orders by (count, node index)). Leaves
// and dummies sit sorted in key[0, items) as count << 11 | index; internal nodes are created
// with non-decreasing counts into q2 (a FIFO), and on equal counts a leaf precedes an internal
// node and an older internal node a younger one. Let smin = the sum of the n smallest live
// counts: every node created from now on has count >= smin, so every live node of count <=
// smin is picked before any new one, n at a time, in sorted order. A round therefore merges a
// window of 32 leaves and 32 internal nodes into one sorted wave (a bitonic merge in registers:
// the internal half is loaded reversed), keeps the prefix of count <= smin (cut at a half's
// last key when more nodes lie beyond it), and creates floor(prefix / n) nodes at once. Window
// keys of internal nodes: count << 11 | (1536 + position in the window): after every leaf on
// equal counts (leaf indices < 1536), in creation order among themselves, distinct.
// r4 ranked the window by binary searches through LDS (~2.2k cycles a round); this round is
// one LDS load, VALU lane moves, and the stores.
static __device__ void huff_merge_wave(const uint64_t *__restrict__ key, uint64_t *__restrict__ q2,
                                       int16_t *__restrict__ parent, int items, int nary, int first_internal,
                                       dc_tree *__restrict__ tree, int *bad)
{
    const int lane = threadIdx.x & 63;
    const bool isL = lane < 32;
    const int j = isL ? lane : 63 - lane;   // the internal half reversed: a bitonic sequence
    // per lane, fixed for every round: its group (lane / n) and place in it (lane % n), and
    // the number of whole groups in lanes 0 .. lane ((lane + 1) / n)
    const int gq = lane / nary, gr = lane - gq * nary, gwhole = (lane + 1) / nary;
    const uint64_t jtag = 1536u + (uint32_t)j;
    int h1 = 0, h2 = 0, t2 = 0, active = items, nxt = first_internal;
    constexpr uint64_t INF = ~0ull;
    while (active > 1) {
        // window: leaves h1 .. h1 + 31 in lanes 0-31, internal nodes h2 + 31 .. h2 in lanes
        // 32-63 (one LDS read per lane, the address chosen by a select)
        const int pos = isL ? h1 + j : h2 + j;
        const bool have = pos < (isL ? items : t2);
        const uint64_t *src = isL ? key : q2;
        const uint64_t raw = src[have ? pos : 0];
        const uint64_t k0 = !have ? INF : isL ? raw : ((raw << 11) | jtag);
        // a half with more nodes beyond the window bounds the prefix at its last window key
        const uint64_t lastL = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(k0 >> 32), 31) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)k0, 31);
        const uint64_t lastQ = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(k0 >> 32), 32) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)k0, 32);
        const uint64_t bound = min(h1 + 32 < items ? lastL : INF, t2 - h2 > 32 ? lastQ : INF);
        const uint64_t k = wave_bitonic_merge(k0, lane);
        const uint64_t cnt = k != INF ? (k >> 11) : 0ull;
        // group sums (a node of this round = lanes kn .. kn + n - 1, summed at lane kn + n - 1)
        // and smin (the n smallest = group 0): n = 2 by one DPP row shift, else a DPP scan less
        // the scan n lanes down
        uint64_t gsum;
        if (nary == 2) {
            const uint32_t plo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)cnt, 0x111, 0xf, 0xf, false);
            const uint32_t phi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(cnt >> 32), 0x111, 0xf, 0xf, false);
            gsum = cnt + (((uint64_t)phi << 32) | plo);   // odd lanes: the pair ending here
        } else {
            const uint64_t S = wave_scan_incl_u64(cnt);
            const int sl = lane >= nary ? lane - nary : lane;
            const uint64_t Sd = (uint64_t)(uint32_t)__shfl((int)(uint32_t)S, sl, 64) |
                                ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(S >> 32), sl, 64) << 32);
            gsum = S - (lane >= nary ? Sd : 0ull);
        }
        const uint64_t smin = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(gsum >> 32), nary - 1) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)gsum, nary - 1);
        // qualifying nodes: a prefix of the lanes (k ascending, INF last)
        const int cq = __popcll(__ballot(k != INF && cnt <= smin && k <= bound));
        int m = cq > 0 ? __builtin_amdgcn_readlane(gwhole, cq - 1) : 0;   // floor(cq / n)
        if (m == 0) { m = 1; *bad = 1; }   // cannot happen: the n smallest always qualify
        const int used = m * nary;
        const bool inB = lane < used;
        const bool leaf = (k & 2047u) < 1536u;
        const int na = __popcll(__ballot(inB && leaf));
        if (inB && gr == nary - 1) q2[t2 + gq] = gsum;
        if (inB) {
            const int node = leaf ? (int)(k & 2047u) : first_internal + h2 + (int)((k & 2047u) - 1536u);
            const int par = nxt + gq;
            if (node < TBL_NODES) parent[node] = (int16_t)par;
            if (tree && gr < 2 && par < TBL_NODES)   // first two children (:978-979)
                (gr ? tree->right : tree->left)[par] = node;
        }
        __builtin_amdgcn_wave_barrier();   // the new nodes' counts are read by the next window
        h1 += na;
        h2 += used - na;
        t2 += m;
        nxt += m;
        active -= m * (nary - 1);
    }
    if (lane == 0 && nxt >= TBL_NODES) *bad = 1;
}

// The table of k_huff_table, by one 256-thread workgroup on the LDS S. With d_total set it
// also writes the encode plan of plan_hist (the histogram of the bytes to be packed): the
// payload bits sum_s plan_hist[s] * nbits[s] (the reference's formula, n_ary_huffman.c:2485)
// and the plan error flag (a byte present without a code), and clears the next plan's slot.
static __device__ void huff_table_body(TblLds &S, const uint64_t *__restrict__ freq, int freq_is_hist256,
                                       const int32_t *__restrict__ lens_in, int M, int nary,
                                       dc_dtable *__restrict__ T, dc_tree *__restrict__ tree,
                                       const uint64_t *plan_hist, uint64_t *__restrict__ d_total,
                                       int *__restrict__ perr, int *__restrict__ perr_next)
{
    uint64_t *const s_key = S.key;
    uint64_t *const s_q2 = S.q2;
    int16_t *const s_parent = S.parent;
    int32_t *const s_len = S.len;
    uint32_t *const s_cnt = S.cnt;
    uint32_t *const s_startv = S.startv;
    uint32_t *const s_starti = S.starti;
    uint32_t *const s_code = S.code;
    uint32_t *const s_nb = S.nb;
    int &s_k = S.k, &s_min = S.mn, &s_max = S.mx, &s_maxbits = S.maxbits, &s_bad = S.bad;

    const int t = threadIdx.x;
    const int leaves = M + 1;
    int w = 0;
    while ((1 << w) < nary) ++w;

    if (t == 0) { s_k = 0; s_min = 300; s_max = 0; s_maxbits = 0; s_bad = 0; }
    __syncthreads();

    if (lens_in == nullptr) {
        for (int i = t; i < leaves; i += 256) {
            const uint64_t f = freq_is_hist256 ? (i < 256 ? freq[i] : 0ull) : freq[i];
            if (f) {
                const int slot = atomicAdd(&s_k, 1);
                s_key[slot] = (f << 11) | (uint64_t)i;
                if (f >> 53) s_bad = 1;
            }
        }
        __syncthreads();
        const int k = s_k;
        const int dummies = (nary - 1) - ((k - 1) % (nary - 1));
        const int items = k + dummies;
        int P = 1;
        while (P < items) P <<= 1;
        for (int i = k + t; i < P; i += 256)
            s_key[i] = (i < items) ? ((1ull << 11) | (uint64_t)(leaves + (i - k))) : ~0ull;
        for (int i = t; i < TBL_NODES; i += 256) s_parent[i] = 0;
        __syncthreads();
        if (items <= 512) {
            // rank sort (keys are distinct: count << 11 | node index): a key's place is the
            // number of keys below it. Every thread reads the same key pair at each step (an
            // LDS broadcast, no conflicts) against its own <= 2 keys: one barrier, ~4 VALU per
            // key pair, where the bitonic network took 36-45 barrier stages (13.4k cycles on C2)
            const uint64_t k0 = t < items ? s_key[t] : ~0ull, k1 = t + 256 < items ? s_key[t + 256] : ~0ull;
            uint32_t r0 = 0, r1 = 0;
            const uint4 *const kp = reinterpret_cast<const uint4 *>(s_key);
            for (int j = 0; j < (items + 1) / 2; ++j) {
                const uint4 q = kp[j];   // keys 2j, 2j + 1 (past items: ~0, never below a key)
                const uint64_t a = ((uint64_t)q.y << 32) | q.x, b = ((uint64_t)q.w << 32) | q.z;
                r0 += (uint32_t)(a < k0) + (uint32_t)(b < k0);
                r1 += (uint32_t)(a < k1) + (uint32_t)(b < k1);
            }
            __syncthreads();
            if (t < items) s_key[r0] = k0;
            if (t + 256 < items) s_key[r1] = k1;
            __syncthreads();
        } else {
            // bitonic sort, ascending
            for (int size = 2; size <= P; size <<= 1) {
                for (int stride = size >> 1; stride > 0; stride >>= 1) {
                    for (int i = t; i < (P >> 1); i += 256) {
                        const int lo = 2 * stride * (i / stride) + (i % stride);
                        const int hi = lo + stride;
                        const bool asc = ((lo & size) == 0);
                        const uint64_t a = s_key[lo], b = s_key[hi];
                        if ((a > b) == asc) { s_key[lo] = b; s_key[hi] = a; }
                    }
                    __syncthreads();
                }
            }
        }
        if (nary <= 32 && t < 64) {
            huff_merge_wave(s_key, s_q2, s_parent, items, nary, leaves + dummies, tree, &s_bad);
        } else if (t == 0) {
            // two-queue merge; both queues' heads and next elements held in registers, the
            // element after them prefetched from LDS when a head is consumed, so no pick
            // waits for an LDS round trip (the internal queue's next element may not exist
            // yet: then it is the sum this step appends, taken from a register)
            int h1 = 0, h2 = 0, t2 = 0, active = items;
            const int first_internal = leaves + dummies;
            int next = first_internal;
            // leaf queue: key[h1 .. h1 + 3] in registers (a 4-deep window refilled from LDS as it
            // moves); internal queue: q2[h2], q2[h2 + 1] in registers
            uint64_t a0 = items > 0 ? s_key[0] : ~0ull, a1 = items > 1 ? s_key[1] : ~0ull;
            uint64_t a2 = items > 2 ? s_key[2] : ~0ull, a3 = items > 3 ? s_key[3] : ~0ull;
            uint64_t head2 = ~0ull, nxt2 = ~0ull;
            while (active > 1) {
                uint64_t sum = 0;
                for (int q = 0; q < nary; ++q) {
                    const uint64_t c1 = (h1 < items) ? (a0 >> 11) : ~0ull;
                    const uint64_t c2 = (h2 < t2) ? head2 : ~0ull;
                    int idx;
                    if (h1 < items && (h2 == t2 || c1 <= c2)) {
                        idx = (int)(a0 & 2047u);
                        sum += c1;
                        ++h1;
                        a0 = a1; a1 = a2; a2 = a3;
                        a3 = (h1 + 3 < items) ? s_key[h1 + 3] : ~0ull;
                    } else {
                        idx = first_internal + h2;
                        sum += c2;
                        ++h2;
                        head2 = nxt2;
                        nxt2 = (h2 + 1 < t2) ? s_q2[h2 + 1] : ~0ull;
                    }
                    if (t == 0 && idx < TBL_NODES) s_parent[idx] = (int16_t)next;
                    if (tree && q < 2 && next < TBL_NODES) (q ? tree->right : tree->left)[next] = idx;
                }
                if (t == 0) s_q2[t2] = sum;
                if (t2 == h2) head2 = sum;            // the queue was empty
                else if (t2 == h2 + 1) nxt2 = sum;   // it held one element
                ++t2;
                ++next;
                active -= nary - 1;
            }
            if (t == 0 && next >= TBL_NODES) s_bad = 1;
        }
        __syncthreads();
        if (tree) {   // the whole node list (generate_huffman_tree's in-out list, :868-1005)
            const int first_internal = leaves + dummies;
            const int nodes = first_internal + max(items - 1, 0) / max(nary - 1, 1);
            for (int i = t; i < TBL_NODES; i += 256) {
                tree->parent[i] = i < nodes ? s_parent[i] : 0;
                uint64_t cnt = 0;
                if (i < leaves) cnt = freq_is_hist256 ? (i < 256 ? freq[i] : 0ull) : freq[i];
                else if (i < first_internal) cnt = 1;   // dummy leaves (:921-929)
                else if (i < nodes) cnt = s_q2[i - first_internal];
                tree->count[i] = cnt;
                if (i >= nodes || i < first_internal) { tree->left[i] = 0; tree->right[i] = 0; }
            }
            if (t == 0) {
                tree->nodes = nodes;
                tree->first_internal = first_internal;
                tree->dummies = dummies;
                tree->status = s_bad ? DC_E_ARG : DC_OK;
            }
        }
        // depth = number of parent hops to the root (n_ary_huffman.c:1069-1076)
        for (int i = t; i < leaves; i += 256) {
            int d = 0, c = i;
            while (s_parent[c] != 0 && d < TBL_NODES) { ++d; c = s_parent[c]; }
            s_len[i] = d;
        }
    } else {
        for (int i = t; i < leaves; i += 256) s_len[i] = lens_in[i];
    }
    // canonical codes (convert_lengths_to_encode_table, :1382-1612): min/max over i < M (:1336),
    // assignment over i <= M. Per length a bitmap of its symbols (in the sort keys' LDS, free
    // now): counts and ranks are popcounts, and the first value per length is one DPP scan of
    // the affine steps code -> (code + cnt) * n. Two barriers where r4's per-wave ballot loops
    // took ten (15k cycles on C2).
    uint32_t *const s_mask = reinterpret_cast<uint32_t *>(s_key);   // [L - 1][32]: symbols of length L
    constexpr int MW = DC_MAX_SYMS / 32;
    static_assert(DC_MAX_DIGITS * MW * sizeof(uint32_t) <= sizeof(S.key), "length bitmaps in the key array");
    for (int q = t; q < DC_MAX_DIGITS * MW / 4; q += 256) reinterpret_cast<uint4 *>(s_mask)[q] = make_uint4(0u, 0u, 0u, 0u);
    {   // min / max length over i < M: per thread, per wave (DPP-free shuffles), one atomic per wave
        int mx = 0, mnl = 300;
        for (int i = t; i < M; i += 256) {
            const int L = s_len[i];
            mx = max(mx, L);
            if (L > 0) mnl = min(mnl, L);
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            mx = max(mx, __shfl_xor(mx, d, 64));
            mnl = min(mnl, __shfl_xor(mnl, d, 64));
        }
        if ((t & 63) == 0) { atomicMax(&s_max, mx); atomicMin(&s_min, mnl); }
    }
    __syncthreads();
    const int minL = s_min, maxL = s_max;
    const int topL = min(maxL, DC_MAX_DIGITS);
    if (maxL > DC_MAX_DIGITS && t == 0) s_bad = 1;
    for (int i = t; i < leaves; i += 256) {
        const int L = s_len[i];
        if (L >= minL && L <= topL) atomicOr(&s_mask[(L - 1) * MW + (i >> 5)], 1u << (i & 31));
    }
    for (int s = t; s < 256; s += 256) { s_code[s] = 0; s_nb[s] = 0; }
    __syncthreads();
    const int nw = (leaves + 31) >> 5;
    if (t < 64) {
        // per length: cnt = popcount of its bitmap; first slot = exclusive sum of the counts;
        // first value (:1540-1568, int arithmetic wrapping mod 2^32) = the composition of the
        // steps f_L(x) = n x + n cnt_L of the lengths below, applied to 0: an exclusive DPP scan
        // of (A, B) pairs (x -> A x + B), carried across blocks of 64 lengths
        uint32_t cin = 0, sin = 0;   // first value and first slot at the block's first length
        for (int base = minL; base <= topL; base += 64) {
            const int L = base + t;
            const bool in = L <= topL;
            uint32_t cl = 0;
            if (in)
                for (int q = 0; q < nw; ++q) cl += (uint32_t)__popc(s_mask[(L - 1) * MW + q]);
            const uint32_t si = wave_scan_incl(cl);
            uint32_t A = in ? (uint32_t)nary : 1u, B = in ? (uint32_t)nary * cl : 0u;
#define DC_AFF_STEP(ctrl, rm)                                                                           \
            {                                                                                           \
                const uint32_t Ae = (uint32_t)__builtin_amdgcn_update_dpp(1, (int)A, ctrl, rm, 0xf, false); \
                const uint32_t Be = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)B, ctrl, rm, 0xf, false); \
                B = A * Be + B;                                                                         \
                A = A * Ae;                                                                             \
            }
            DC_AFF_STEP(0x111, 0xf) DC_AFF_STEP(0x112, 0xf) DC_AFF_STEP(0x114, 0xf) DC_AFF_STEP(0x118, 0xf)
            DC_AFF_STEP(0x142, 0xa) DC_AFF_STEP(0x143, 0xc)
#undef DC_AFF_STEP
            // exclusive: the inclusive pair of the lane below (identity at lane 0)
            const uint32_t Ax = (uint32_t)__builtin_amdgcn_update_dpp(1, (int)A, 0x138, 0xf, 0xf, false);   // wave_shr:1
            const uint32_t Bx = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)B, 0x138, 0xf, 0xf, false);
            if (in) {
                s_cnt[L] = cl;
                s_startv[L] = Ax * cin + Bx;
                s_starti[L] = sin + si - cl;
            }
            const uint32_t A63 = (uint32_t)__builtin_amdgcn_readlane((int)A, 63), B63 = (uint32_t)__builtin_amdgcn_readlane((int)B, 63);
            cin = A63 * cin + B63;
            sin += (uint32_t)__builtin_amdgcn_readlane((int)si, 63);
        }
        for (int L = t; L < minL && L <= DC_MAX_DIGITS; L += 64) { s_cnt[L] = 0; s_startv[L] = 0; s_starti[L] = 0; }
        for (int L = topL + 1 + t; L <= DC_MAX_DIGITS; L += 64) {
            if (L >= minL) { s_cnt[L] = 0; s_startv[L] = 0; s_starti[L] = sin; }
        }
    }
    __syncthreads();
    for (int i = t; i < leaves; i += 256) {
        // canonical rank = symbols of the same length before this one (index order)
        const int L = s_len[i];
        const bool coded = L >= minL && L <= topL;
        T->lengths[i] = L;
        if (coded) {
            const uint32_t *mk = s_mask + (L - 1) * MW;
            uint32_t rank = (uint32_t)__popc(mk[i >> 5] & ((1u << (i & 31)) - 1u));
            for (int q = 0; q < (i >> 5); ++q) rank += (uint32_t)__popc(mk[q]);
            const uint32_t val = s_startv[L] + rank;
            T->enc_len[i] = L;
            T->enc_val[i] = val;
            T->syms[s_starti[L] + rank] = (uint16_t)i;
            if (i < 256) {
                // L base-n digits of val, MSB-first, w bits each (n = 2^w: the bits of val)
                if ((long long)L * w <= 32) {
                    uint32_t v = val;
                    uint64_t packed = 0;
                    if ((nary & (nary - 1)) == 0) {
                        packed = (L * w >= 32) ? (uint64_t)val : ((uint64_t)val & ((1ull << (L * w)) - 1));
                    } else {
                        for (int d = 0; d < L; ++d) {
                            packed |= (uint64_t)(v % (uint32_t)nary) << (w * d);
                            v /= (uint32_t)nary;
                        }
                    }
                    s_code[i] = (uint32_t)packed;
                    s_nb[i] = (uint32_t)(L * w);
                    atomicMax(&s_maxbits, L * w);
                } else {
                    atomicMax(&s_maxbits, 33);
                }
            }
            if (i == M) T->last_written = 1;
        } else {
            if (i < M) { T->enc_len[i] = 0; T->enc_val[i] = 0; }
            else { T->last_written = 0; T->enc_len[i] = 0; T->enc_val[i] = 0; }
        }
    }
    for (int i = leaves + t; i < DC_MAX_SYMS; i += 256) {
        T->lengths[i] = 0; T->enc_len[i] = 0; T->enc_val[i] = 0;
    }
    for (int L = t; L <= DC_MAX_DIGITS; L += 256) {
        const bool in = (L >= minL && L <= maxL);
        T->first[L] = in ? s_startv[L] : 0u;
        T->count[L] = in ? s_cnt[L] : 0u;
        T->start[L] = s_starti[L];
    }
    // left-justified canonical limits per BIT length b (power-of-two n): codes of digit
    // length <= floor(b/w) are exactly the 32-bit windows below lim[b]
    if (t <= 32) {
        const int Ld = t / w;
        uint64_t lim;
        if (Ld < minL) lim = 0;
        else if (Ld >= maxL || Ld * w > 32) lim = 1ull << 32;
        else lim = ((uint64_t)s_startv[Ld] + s_cnt[Ld]) << (32 - Ld * w);
        T->lim[t] = lim;
    }
    __syncthreads();   // s_code, s_nb, s_maxbits
    T->code[t] = s_code[t];
    T->nbits[t] = s_nb[t];
    // every coded byte 8 bits long (n = 16 on a flat byte distribution: a full depth-2 tree):
    // pack and decode become byte maps (k_huff_pack / k_huff_decode8 fast paths)
    const int fixed_ok = __syncthreads_and(s_nb[t] == 0u || s_nb[t] == 8u);
    const int fixed_any = __syncthreads_or(s_nb[t] == 8u);
    // affine: the codes of one length count up from 0 in byte order (canonical), so they are
    // byte - lo exactly when the coded bytes are one run lo .. lo + count - 1
    if (t == 0) S.aff_lo = -1;
    const int ncoded = __syncthreads_count(s_nb[t] == 8u);
    if (s_nb[t] == 8u && s_code[t] == 0u) S.aff_lo = t;
    __syncthreads();
    const int aff_lo = S.aff_lo;
    const int affine = __syncthreads_and(s_nb[t] != 8u || (aff_lo >= 0 && s_code[t] == (uint32_t)(t - aff_lo)));
    if (t == 0) {
        T->fixed8 = (fixed_ok && fixed_any) ? 1 : 0;
        T->fixed8_affine = (fixed_ok && fixed_any && affine) ? 1 : 0;
        T->fixed8_lo = aff_lo;
        T->fixed8_count = ncoded;
        T->n_ary = nary;
        T->w = w;
        T->max_symbol_value = M;
        T->max_bits = s_maxbits;
        T->min_len = minL;
        T->max_len = maxL;
        T->dec_ready = 0;   // the decoder tables follow (k_huff_pack's builder, or k_dec_tables)
        T->status = s_bad ? DC_E_ARG : (s_maxbits > 32 ? DC_E_CODE_TOO_LONG : DC_OK);
    }
    if (d_total) {   // the plan: payload bits of plan_hist under this code, missing codes
        const uint64_t h = plan_hist[t];
        const uint32_t nb = s_nb[t];
        uint64_t v = h * nb;
        const bool miss = h != 0 && nb == 0;
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
        const bool anymiss = __syncthreads_or(miss);
        if ((t & 63) == 0) S.red[t >> 6] = v;
        __syncthreads();
        if (t == 0) {
            *d_total = S.red[0] + S.red[1] + S.red[2] + S.red[3];
            perr[0] = anymiss ? 1 : 0;
        }
        if (t < 4) perr_next[t] = 0;   // the next plan's error slot
    }
}

__global__ __launch_bounds__(256) void k_huff_table(const uint64_t *__restrict__ freq, int freq_is_hist256,
                                                    const int32_t *__restrict__ lens_in, int M, int nary,
                                                    dc_dtable *__restrict__ T, dc_tree *__restrict__ tree,
                                                    const uint64_t *__restrict__ plan_hist, uint64_t *__restrict__ d_total,
                                                    int *__restrict__ perr, int *__restrict__ perr_next)
{
    __shared__ TblLds S;
    huff_table_body(S, freq, freq_is_hist256, lens_in, M, nary, T, tree, plan_hist, d_total, perr, perr_next);
}

// dc_huff_plan: the encode plan of this context's last histogram under a table built elsewhere
// (the multi-rank paths: the table comes from the all-reduced or broadcast histogram)
__global__ __launch_bounds__(256) void k_plan_total(const uint64_t *__restrict__ plan_hist, const dc_dtable *__restrict__ T,
                                                    uint64_t *__restrict__ d_total, int *__restrict__ perr,
                                                    int *__restrict__ perr_next)
{
    __shared__ uint64_t red[4];
    const int t = threadIdx.x;
    const uint64_t h = plan_hist[t];
    const uint32_t nb = T->nbits[t];
    uint64_t v = h * nb;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    const bool anymiss = __syncthreads_or(h != 0 && nb == 0);
    if ((t & 63) == 0) red[t >> 6] = v;
    __syncthreads();
    if (t == 0) {
        *d_total = red[0] + red[1] + red[2] + red[3];
        perr[0] = anymiss ? 1 : 0;
    }
    if (t < 4) perr_next[t] = 0;
}

// ------------------------------------------------------------------------------------
// Decoder tables of a code table (dc_gpu.h: lut, dlut, dlut2, dlut14, dlut15), built by one
// 256-thread workgroup from the canonical arrays k_huff_table wrote. Not on the encoder's
// critical path: k_huff_pack runs it in an extra workgroup beside the pack (its LDS is the
// pack stage), and dc_huff_decode launches k_dec_tables first, which returns at once when the
// tables are current (dec_ready). 55k of k_huff_table's 184k cycles moved off the encode (r2).
// ------------------------------------------------------------------------------------
struct DecBuildLds {
    uint32_t lut1[1 << DC_LUT_BITS];   // one-symbol table, MSB-first 12-bit window -> sym | nbits << 8
    uint16_t esc[1 << DC_LUT_BITS];    // escape id per dlut entry
    uint32_t code[256], nb[256];
    uint32_t startv[DC_MAX_DIGITS + 2], cnt[DC_MAX_DIGITS + 2], starti[DC_MAX_DIGITS + 2];
    uint16_t syms[DC_MAX_SYMS];
    uint32_t tot_esc[256];
    int nesc;
};

static __device__ void dec_tables_build(dc_dtable *__restrict__ T, DecBuildLds &S)
{
    const int t = threadIdx.x;
    const int nary = T->n_ary, w = T->w, minL = T->min_len, maxL = T->max_len, maxbits = T->max_bits;
    S.code[t] = T->code[t];
    S.nb[t] = T->nbits[t];
    for (int L = t; L < DC_MAX_DIGITS + 1; L += 256) {
        S.startv[L] = T->first[L];
        S.cnt[L] = T->count[L];
        S.starti[L] = T->start[L];
    }
    for (int i = t; i < DC_MAX_SYMS; i += 256) S.syms[i] = T->syms[i];
    for (int e = t; e < (1 << DC_LUT_BITS); e += 256) S.lut1[e] = 0;
    __syncthreads();
    uint32_t *const s_lut1 = S.lut1;
    if ((nary & (nary - 1)) == 0) {
        // n = 2^w: a 12-bit window's code is the canonical one whose value at its length
        // matches (lengths ascending), decoded per entry
        for (int e = t; e < (1 << DC_LUT_BITS); e += 256) {
            uint32_t v1 = 0;
            for (int L = minL; L <= maxL && L * w <= DC_LUT_BITS; ++L) {
                const uint32_t b = (uint32_t)(L * w), v = (uint32_t)e >> (DC_LUT_BITS - b);
                if (v - S.startv[L] < S.cnt[L]) {
                    const uint32_t sym = S.syms[(S.starti[L] + v - S.startv[L]) & (DC_MAX_SYMS - 1)];
                    v1 = sym < 256 ? (sym | (b << 8)) : 0u;
                    break;
                }
            }
            s_lut1[e] = v1;
        }
    } else {   // thread s fills its own code's span
        const uint32_t nb = S.nb[t];
        if (nb != 0 && nb <= DC_LUT_BITS) {
            const uint32_t span = 1u << (DC_LUT_BITS - nb);
            const uint32_t base = S.code[t] << (DC_LUT_BITS - nb);
            for (uint32_t j = 0; j < span; ++j) s_lut1[base + j] = (uint32_t)t | (nb << 8);
        }
    }
    __syncthreads();
    // two-symbol table: a window holding a whole second code after the first yields both
    // (DC_LUT_* layout in dc_gpu.h)
    for (int e = t; e < (1 << DC_LUT_BITS); e += 256) {
        const uint32_t a = s_lut1[e];
        uint32_t v = 0;
        if (a) {
            const uint32_t s0 = a & 255u, n0 = a >> 8;
            v = s0 | (n0 << 8) | (n0 << 24) | (1u << 29);
            const uint32_t b = s_lut1[((uint32_t)e << n0) & ((1u << DC_LUT_BITS) - 1)];
            if (b && (b >> 8) <= DC_LUT_BITS - n0)
                v = s0 | ((n0 + (b >> 8)) << 8) | ((b & 255u) << 16) | (n0 << 24) | (2u << 29);
        }
        T->lut[e] = v;
    }
    // decoder tables on the LSB-first window (dc_gpu.h): dlut = the one-symbol table at the
    // bit-reversed index; escape prefixes (entries 0) numbered in index order; dlut2 filled
    // per symbol: a code of 12 < b <= 12 + k bits covers 2^(12 + k - b) entries of its
    // prefix's sub-table (no per-entry search)
    uint16_t *const s_esc = S.esc;
    constexpr int PER = (1 << DC_LUT_BITS) / 256;
    uint32_t d1[PER], nesc = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t i = (uint32_t)(t * PER + j);
        const uint32_t a = s_lut1[__builtin_bitreverse32(i) >> (32 - DC_LUT_BITS)];
        d1[j] = a ? ((a >> 8) | ((a & 255u) << 8)) : 0u;
        nesc += a ? 0u : 1u;
    }
    {   // exclusive scan of the per-thread escape counts: DPP inside each wave, 4 wave totals
        const uint32_t inc = wave_scan_incl(nesc);
        if ((t & 63) == 63) S.tot_esc[t >> 6] = inc;
        __syncthreads();
        uint32_t before = 0, all = 0;
        for (int q = 0; q < 4; ++q) {
            const uint32_t v = S.tot_esc[q];
            before += (q < (t >> 6)) ? v : 0u;
            all += v;
        }
        __syncthreads();
        S.tot_esc[t] = before + inc - nesc;
        if (t == 0) S.nesc = (int)all;   // escape prefixes
        __syncthreads();
    }
    const uint32_t E = (uint32_t)S.nesc;
    const uint32_t K = (uint32_t)min(max(maxbits - DC_LUT_BITS, 1), 8);
    const bool l2ok = E > 0 && E <= 256 && (E << K) <= DC_LUT2_CAP && maxbits <= 32;
    uint32_t id = S.tot_esc[t];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t i = (uint32_t)(t * PER + j);
        uint32_t v = d1[j];
        if (!v) { s_esc[i] = (uint16_t)id; v = (id & 255u) << 8; ++id; }
        T->dlut[i] = (uint16_t)v;
    }
    for (int q = t; q < DC_LUT2_CAP; q += 256) T->dlut2[q] = 0;
    __syncthreads();   // s_esc complete; dlut2 zeroed (same workgroup: global writes ordered by the barrier)
    if (l2ok) {
        const uint32_t nb = S.nb[t];
        if (nb > DC_LUT_BITS && nb <= DC_LUT_BITS + K) {
            const uint32_t c = S.code[t], tl = nb - DC_LUT_BITS;
            const uint32_t pre = __builtin_bitreverse32(c >> tl) >> (32 - DC_LUT_BITS);   // first 12 stream bits
            const uint32_t rt = __builtin_bitreverse32(c & ((1u << tl) - 1)) >> (32 - tl);
            const uint32_t base = (uint32_t)s_esc[pre] << K;
            for (uint32_t j = 0; j < (1u << (K - tl)); ++j) T->dlut2[base | rt | (j << tl)] = (uint16_t)(nb | ((uint32_t)t << 8));
        }
    }
    __syncthreads();   // dlut2 complete
    // dlut14 and dlut15, two entries per u32 store (coalesced): entry x = dlut entry x & 4095
    // (from s_lut1, as d1 above), an escape there resolved on the next 2 (3) bits by dlut2
    // when that code fits 14 (15) bits
    // zesc: an entry of no code in the table is 0 (the fast decoder tests min(entry) == 0)
    // instead of carrying the escape id
    auto wide = [&](uint16_t *dst, uint32_t bits, bool zesc) {
        const bool l2w = l2ok && K >= bits - DC_LUT_BITS;
        uint32_t *const dw = reinterpret_cast<uint32_t *>(dst);
#pragma unroll 8
        for (uint32_t p = t; p < (1u << bits) / 2; p += 256) {
            uint32_t pr = 0;
#pragma unroll
            for (uint32_t q = 0; q < 2; ++q) {
                const uint32_t x = 2 * p + q, i = x & ((1u << DC_LUT_BITS) - 1), h = x >> DC_LUT_BITS;
                const uint32_t a = s_lut1[__builtin_bitreverse32(i) >> (32 - DC_LUT_BITS)];
                uint32_t e = (a >> 8) | ((a & 255u) << 8);
                if (!a) {
                    const uint32_t esc = s_esc[i];
                    const uint32_t e2 = l2w ? T->dlut2[(esc << K) | h] : 0u;
                    e = (e2 && (e2 & 255u) <= bits) ? e2 : zesc ? 0u : ((esc & 255u) << 8);
                }
                pr |= e << (16 * q);
            }
            dw[p] = pr;
        }
    };
    wide(T->dlut14, DC_LUT14_BITS, false);
    wide(T->dlut15, DC_LUT15_BITS, true);
    if (t == 0) T->dlut2_k = l2ok ? (int32_t)K : 0;
    __syncthreads();
    if (t == 0) {   // every table store of the workgroup before the flag (agent scope)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_store(&T->dec_ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// dc_huff_decode's first launch: the decoder tables unless they are current
__global__ __launch_bounds__(256) void k_dec_tables(dc_dtable *__restrict__ T, int *__restrict__ err_clear)
{
    __shared__ DecBuildLds S;
    if (threadIdx.x == 0) err_clear[0] = 0;
    if (__hip_atomic_load(&T->dec_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || T->status != DC_OK) return;
    dec_tables_build(T, S);
}

// summarize_tree_with_lengths (n_ary_huffman.c:1033-1093) for an arbitrary node list:
// depth of node i < leaves = parent hops up to the node whose parent is 0, minus one (the
// root); a walk longer than the list (a cycle) reports -1
__global__ void k_tree_depths(const int32_t *__restrict__ parent, int list_length, int leaves,
                              int32_t *__restrict__ depth)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= leaves) return;
    int c = i, sum = 0;
    do {
        ++sum;
        c = (c >= 0 && c < list_length) ? parent[c] : 0;
    } while (c != 0 && sum <= list_length);
    depth[i] = sum > list_length ? -1 : sum - 1;
}

// ------------------------------------------------------------------------------------
// (H7) encode plan: bits per 32 KiB block = sum_s h_b[s] * nbits[s] (the reference's
// own payload formula, n_ary_huffman.c:2485), then an exclusive scan over blocks.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_block_bits(const uint16_t *__restrict__ bh, uint64_t nblocks,
                                                    const dc_dtable *__restrict__ T,
                                                    uint64_t *__restrict__ bits, int *__restrict__ err)
{
    const int lane = threadIdx.x & 63;
    const uint64_t b = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= nblocks) return;
    const uint2 h = *reinterpret_cast<const uint2 *>(bh + b * 256 + lane * 4);
    const uint32_t c[4] = {h.x & 0xFFFFu, h.x >> 16, h.y & 0xFFFFu, h.y >> 16};
    uint64_t acc = 0;
    int missing = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t nb = T->nbits[lane * 4 + j];
        acc += (uint64_t)c[j] * nb;
        missing |= (c[j] != 0 && nb == 0);
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) acc += __shfl_xor(acc, d, 64);
    if (__any(missing) && lane == 0) atomicOr(err, 1);
    if (lane == 0) bits[b] = acc;
}

// single-workgroup exclusive scan; off[b] relative, off[nblocks] = total
__global__ __launch_bounds__(1024) void k_block_scan(uint64_t *__restrict__ bits_off, uint64_t nblocks,
                                                     uint64_t *__restrict__ d_total, int *__restrict__ err_next)
{
    __shared__ uint64_t s[1024];
    const int t = threadIdx.x;
    if (t < 4) err_next[t] = 0;   // the next plan's error slot
    const uint64_t per = (nblocks + 1023) / 1024;
    const uint64_t b0 = (uint64_t)t * per;
    const uint64_t b1 = (b0 + per < nblocks) ? b0 + per : nblocks;
    uint64_t sum = 0;
    uint64_t b = b0;
    for (; b + 8 <= b1; b += 8) {   // 8 independent loads in flight per lane
        uint64_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = bits_off[b + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) sum += v[k];
    }
    for (; b < b1; ++b) sum += bits_off[b];
    s[t] = sum;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const uint64_t y = (t >= d) ? s[t - d] : 0ull;
        __syncthreads();
        s[t] += y;
        __syncthreads();
    }
    uint64_t run = s[t] - sum;
    b = b0;
    for (; b + 8 <= b1; b += 8) {
        uint64_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = bits_off[b + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) { bits_off[b + k] = run; run += v[k]; }
    }
    for (; b < b1; ++b) {
        const uint64_t v = bits_off[b];
        bits_off[b] = run;
        run += v;
    }
    if (t == 1023) {
        bits_off[nblocks] = s[1023];
        *d_total = s[1023];
    }
}

// Plan in two launches (k_block_bits + the single-workgroup k_block_scan read 32768
// offsets with strided, uncoalesced loads: 40 us on 1 GiB): (1) a workgroup per 64 blocks
// computes their bit counts and scans them locally; (2) a workgroup per 64 blocks adds the
// workgroup totals before it and writes its blocks' absolute offsets.
#define PLAN_WG_BLOCKS 64
#define PLAN_MAX_WG 16384   /* workgroup bases in LDS (128 KiB): streams up to 32 GiB per call */
// With lcnt set (the C5 fused front-end, whose blocks hold a varying number of symbols) it
// also scans the symbols per block (the sum of its histogram) into lcnt / wgcnt.
__global__ __launch_bounds__(256) void k_block_local(const uint16_t *__restrict__ bh, uint64_t nblocks,
                                                     const dc_dtable *__restrict__ T, uint32_t *__restrict__ local,
                                                     uint32_t *__restrict__ wgtot, int *__restrict__ err,
                                                     uint32_t *__restrict__ lcnt, uint32_t *__restrict__ wgcnt)
{
    __shared__ uint32_t s_nb[256];
    __shared__ uint32_t s_bits[PLAN_WG_BLOCKS];
    __shared__ uint32_t s_syms[PLAN_WG_BLOCKS];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    s_nb[t] = T->nbits[t];
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * PLAN_WG_BLOCKS;
    int missing = 0;
    // all 16 of the wave's block-histogram loads in flight at once
    uint2 hv[PLAN_WG_BLOCKS / 4];
#pragma unroll
    for (int k = 0; k < PLAN_WG_BLOCKS / 4; ++k) {
        const uint64_t b = b0 + wv * (PLAN_WG_BLOCKS / 4) + k;
        hv[k] = b < nblocks ? *reinterpret_cast<const uint2 *>(bh + b * 256 + lane * 4) : make_uint2(0u, 0u);
    }
#pragma unroll
    for (int k = 0; k < PLAN_WG_BLOCKS / 4; ++k) {
        const int j = wv * (PLAN_WG_BLOCKS / 4) + k;
        const uint64_t b = b0 + j;
        uint32_t acc = 0, syms = 0;
        if (b < nblocks) {
            const uint2 h = hv[k];
            const uint32_t c[4] = {h.x & 0xFFFFu, h.x >> 16, h.y & 0xFFFFu, h.y >> 16};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t nb = s_nb[lane * 4 + q];
                acc += c[q] * nb;
                syms += c[q];
                missing |= (c[q] != 0 && nb == 0);
            }
        }
        acc = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_incl(acc), 63);   // <= 2^20 per block
        if (lane == 0) s_bits[j] = acc;
        if (lcnt) {
            syms = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_incl(syms), 63);
            if (lane == 0) s_syms[j] = syms;
        }
    }
    if (__any(missing) && lane == 0) atomicOr(err, 1);
    __syncthreads();
    if (wv == 0) {
        const uint32_t v = s_bits[lane];
        const uint32_t incl = wave_scan_incl(v);   // <= 2^26 per workgroup
        if (b0 + lane < nblocks) local[b0 + lane] = incl - v;
        if (lane == 63) wgtot[blockIdx.x] = incl;
    } else if (wv == 1 && lcnt) {
        const uint32_t v = s_syms[lane];
        const uint32_t incl = wave_scan_incl(v);   // <= 2^21 per workgroup
        if (b0 + lane < nblocks) lcnt[b0 + lane] = incl - v;
        if (lane == 63) wgcnt[blockIdx.x] = incl;
    }
}

// (2), one workgroup per PLAN_WG_BLOCKS blocks: its base = the sum of the workgroup totals
// before it (every workgroup re-reads the <= PLAN_MAX_WG totals: 2 KiB on 1 GiB), then its
// blocks' absolute offsets; the last workgroup writes the stream total
// With `words` set it also zeroes every word two blocks share (the word holding a block's
// first bit, and the stream's partial last word), which k_huff_pack OR-merges into: words
// whose index is past words_cap are left alone (the pack reports the capacity error).
__global__ __launch_bounds__(256) void k_block_final_wide(const uint32_t *__restrict__ local,
                                                          const uint32_t *__restrict__ wgtot, uint64_t nblocks,
                                                          uint32_t nwg, uint64_t *__restrict__ off,
                                                          uint64_t *__restrict__ d_total, int *__restrict__ err_next,
                                                          uint64_t bit_base, const uint64_t *__restrict__ d_base,
                                                          uint32_t *__restrict__ words, uint64_t words_cap,
                                                          const uint32_t *__restrict__ lcnt,
                                                          const uint32_t *__restrict__ wgcnt, uint64_t *__restrict__ msym,
                                                          uint32_t *__restrict__ sl32, uint32_t slog,
                                                          const int64_t *__restrict__ shard = nullptr,
                                                          uint32_t *__restrict__ gl32 = nullptr)
{
    // With lcnt set (C5 fused front-end): msym[b] = the index of block b's first symbol
    // (msym[nblocks] = all symbols), and the sync-length dword holding the chunk that spans each
    // block boundary (the last chunk begun before block b, b = 1..nblocks) is zeroed: k_fe_pack
    // adds the two blocks' parts of it, and of its dword neighbour, atomically.
    __shared__ uint64_t s_w[4], s_c[4];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t g = blockIdx.x;
    if (g == 0 && t < 4) err_next[t] = 0;   // the next plan's error slot
    const bool last = g + 1 == nwg;
    const uint32_t lim = last ? nwg : g;   // the last workgroup sums everything (the total)
    uint64_t before = 0, all = 0, cbefore = 0, call = 0;
    for (uint32_t i = t; i < lim; i += 256) {
        const uint64_t v = wgtot[i];
        all += v;
        before += i < g ? v : 0ull;
        if (lcnt) {
            const uint64_t cv = wgcnt[i];
            call += cv;
            cbefore += i < g ? cv : 0ull;
        }
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        before += __shfl_xor(before, d, 64);
        all += __shfl_xor(all, d, 64);
        if (lcnt) {
            cbefore += __shfl_xor(cbefore, d, 64);
            call += __shfl_xor(call, d, 64);
        }
    }
    if (lane == 0) { s_w[wv] = before; s_c[wv] = cbefore; }
    __syncthreads();
    const uint64_t base = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    const uint64_t cbase = s_c[0] + s_c[1] + s_c[2] + s_c[3];
    __syncthreads();
    if (lcnt) {
        if (lane == 0) s_c[wv] = call;
        __syncthreads();
        const uint64_t ctot = s_c[0] + s_c[1] + s_c[2] + s_c[3];
        // (a shard, gl32 set: the same dwords of its global sync index, whose first chunk is also
        // shared, with the previous shard; k_fe_pack<true>)
        const uint64_t M = gl32 ? (uint64_t)shard[1] : 0, c0e = (M >> slog) & ~1ull;
        auto zero_g = [&](uint64_t m) {
            if (gl32 && M + m > 0 && ((M + m - 1) >> slog) >= c0e) gl32[(((M + m - 1) >> slog) - c0e) >> 1] = 0u;
        };
        if (t < PLAN_WG_BLOCKS) {
            const uint64_t b = (uint64_t)g * PLAN_WG_BLOCKS + t;
            if (b < nblocks) {
                const uint64_t m = cbase + lcnt[b];
                msym[b] = m;
                if (b > 0) sl32[((m - 1) >> slog) >> 1] = 0u;
                zero_g(m);
            }
        } else if (t == PLAN_WG_BLOCKS && last) {
            msym[nblocks] = ctot;
            sl32[((ctot - 1) >> slog) >> 1] = 0u;
            zero_g(ctot);
        }
    }
    if (last) {
        if (lane == 0) s_w[wv] = all;
        __syncthreads();
        if (t == 0) {
            const uint64_t tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
            off[nblocks] = tot;
            *d_total = tot;
        }
    }
    if (d_base) bit_base += *d_base;   // device-resident shard offset (dist: no host read)
    if (t < PLAN_WG_BLOCKS) {
        const uint64_t b = (uint64_t)g * PLAN_WG_BLOCKS + t;
        if (b < nblocks) {
            const uint64_t o = base + local[b];
            off[b] = o;
            const uint64_t wi = ((bit_base + o) >> 5) - (bit_base >> 5);
            if (words && wi < words_cap) words[wi] = 0u;
        }
    } else if (t == PLAN_WG_BLOCKS && last && words) {   // the stream's partial last word
        const uint64_t abs = bit_base + s_w[0] + s_w[1] + s_w[2] + s_w[3];
        const uint64_t wi = (abs >> 5) - (bit_base >> 5);
        if ((abs & 31) != 0 && wi < words_cap) words[wi] = 0u;
    }
}

// ------------------------------------------------------------------------------------
// (H7) pack. One workgroup per 32 KiB block (grid-stride), 8 tiles of 4 KiB; a lane
// codes 16 bytes (one 16-B load). Per tile: LDS table lookups -> workgroup scan of bit
// counts -> each lane writes its bits into an LDS staging area of 32-bit words
// (ds_or_b32 only for the words it shares with a neighbour lane) -> coalesced dword
// stores of the complete words; the partial last word is carried to the next tile.
// Only the two words a block shares with its neighbour blocks are OR-ed into HBM with
// global atomics. The stream is MSB-first: staged words are byte-swapped on store.
// ------------------------------------------------------------------------------------
// A workgroup barrier that orders LDS only (the pack's barriers order its LDS stage). (A
// prefetch of the next block by LDS-DMA, issued after the stage atomics, measured 10% slower.)
static __device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

#define PACK_TILE 4096
#define D8_WSCR (2 * 4096 + 66 * 8 + 512)            /* per-wave scratch of the decoders (bytes)  */
#define D8_SCRATCH_WAVES 4096                        /* waves with a scratch slot (decoders, pack trash rows) */
#define PACK_STAGE (PACK_TILE + 64)
#define PACK_BLK_WORDS 9216     /* 36 KiB: a full block of <= 9 bits/symbol is staged whole  */
#define PACK_PIECES (DC_BLOCK_BYTES / PACK_TILE)

// zero every word two blocks share (plan fallback above PLAN_MAX_WG workgroups of blocks,
// where k_block_final_wide does not run)
__global__ void k_zero_bounds(const uint64_t *__restrict__ off, uint64_t nblocks, uint64_t bit_base,
                              const uint64_t *__restrict__ d_base, uint32_t *__restrict__ words, uint64_t words_cap)
{
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d_base) bit_base += *d_base;
    if (b > nblocks) return;
    const uint64_t abs = bit_base + off[b], wi = (abs >> 5) - (bit_base >> 5);
    if ((b < nblocks || (abs & 31) != 0) && wi < words_cap) words[wi] = 0u;
}

// The pack's block offsets come from the two plan kernels (k_block_local, k_block_final_wide,
// which also zeroes the words two blocks share). (r3 measured the alternatives in one launch:
// a decoupled look-back over pairs of blocks claimed from a counter, 0.60-0.70 ms on 1 GiB C2,
// and over ranges of 4-16 blocks per workgroup, 0.45-0.50 ms, against 0.373 for this pack after
// the plan launches: a look-back costs ~2 us per agent-scope round trip, and ranges of blocks
// long enough to hide it leave the last dispatch round unbalanced.)
template <bool PF = false>   // PF (A/B): the next block loaded piece by piece as pass B frees each
__global__ __launch_bounds__(256) void k_huff_pack(const uint8_t *__restrict__ in, uint64_t n,
                                                   const dc_dtable *__restrict__ T,
                                                   const uint64_t *__restrict__ block_off, uint64_t bit_base,
                                                   const uint64_t *__restrict__ d_base, uint32_t *__restrict__ out, uint64_t *__restrict__ sync_base,
                                                   uint16_t *__restrict__ sync_len, uint32_t sync_syms,
                                                   uint64_t nblocks, uint64_t words_cap,
                                                   int *__restrict__ err, int build_dec)
{
    __shared__ uint2 s_tab[256];
    // bit lengths alone (pass A reads 1 byte, not 8): 64 dwords, so at most 2 distinct dwords
    // per bank. (As dwords, one SDWA shift per byte instead of an extract and a mask, pass A
    // had 256 dwords, 8 per bank: the bank conflicts cost more than the VALU saved, C4 pack +2%;
    // one lookup per byte with the codes held in registers through the scan, in two groups
    // of 4 pieces to fit 128 VGPRs, measured equal on C2 and +3% on C4.)
    __shared__ uint8_t s_nb8[256];
    __shared__ __attribute__((aligned(16))) uint32_t s_stage[PACK_BLK_WORDS + 4];   // +4: emit's no-op ORs past the end
    __shared__ uint32_t s_scan[4];
    __shared__ uint32_t s_tot[PACK_PIECES][4];
    static_assert(sizeof(DecBuildLds) <= sizeof(s_stage), "decoder-table builder uses the stage");
    const int t = threadIdx.x;
    if (build_dec && blockIdx.x == 0) {   // workgroup 0: the decoder tables, beside the pack
        if (T->status == DC_OK)
            dec_tables_build(const_cast<dc_dtable *>(T), *reinterpret_cast<DecBuildLds *>(s_stage));
        return;
    }
    const uint64_t bx = blockIdx.x - (uint64_t)build_dec, gstride = gridDim.x - (uint64_t)build_dec;
    if (d_base) bit_base += *d_base;   // device-resident shard offset (dist: no host read)
    // device-side guards (no host round trip): a byte without a code (plan error) or an
    // output buffer smaller than the planned stream -> write nothing
    const uint64_t total = block_off[nblocks];
    if (err[0] != 0) return;
    if (((bit_base & 31) + total + 31) / 32 > words_cap) {
        if (t == 0) err[2] = 1;   // (pack status: DC_E_CAPACITY)
        return;
    }
    s_tab[t] = make_uint2(T->code[t], T->nbits[t]);
    s_nb8[t] = (uint8_t)T->nbits[t];
    const bool vec_out = ((uintptr_t)out & 15) == 0;
    const uint64_t word_base = bit_base >> 5;
    const uint32_t slog = sync_syms ? (uint32_t)__builtin_ctz(sync_syms) : 0u;   // S is a power of two
    // quarter mode (uniform): above 5.5 bits per symbol on average a fair share of 8-code
    // halves exceed 64 bits, and a wave with one such lane ran both the half and the quarter
    // path; such streams (e.g. C4's Zipf bytes, 6.25) code every half as two quarters
    const bool qmode = 2 * total > 11 * n;
    // the stage is all zero at every block start (each block zeroes what it used)
    for (uint32_t i = 4u * t; i < PACK_BLK_WORDS + 4; i += 1024u)
        *reinterpret_cast<uint4 *>(&s_stage[i]) = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    if (T->fixed8 && vec_out && (bit_base & 127) == 0) {
        // every code 8 bits: stream byte bit_base / 8 + i = code(in[i]) (bit_base % 128 == 0: the
        // stream's first byte is out's first byte, 16-B aligned); the plan is 8 bits per byte.
        // (A byte without a code is the plan's error, found from the histogram before the pack.)
        uint8_t *const ob = reinterpret_cast<uint8_t *>(out);
        for (uint64_t b = bx; b < nblocks; b += gstride) {
            const uint64_t blk_start = b * (uint64_t)DC_BLOCK_BYTES;
            const uint64_t blk_end = (blk_start + DC_BLOCK_BYTES < n) ? blk_start + DC_BLOCK_BYTES : n;
            if (blk_start + DC_BLOCK_BYTES <= n) {
                uint4 v[PACK_PIECES];
#pragma unroll
                for (int k = 0; k < PACK_PIECES; ++k)
                    v[k] = LD_PACK(reinterpret_cast<const uint4 *>(in + blk_start + (uint64_t)k * PACK_TILE + (uint64_t)t * 16));
                // (the affine map, code = byte - lo, is one subtraction per dword here, and measured
                // slower than these lookups: 0.444 vs 0.358 ms per GiB of C3,
                // profiles/r6r_fixed8_affine_ab.log; only the decoder uses it)
#pragma unroll
                for (int k = 0; k < PACK_PIECES; ++k) {
                    uint32_t w4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint32_t x = w4[q];
                        w4[q] = s_tab[x & 255u].x | (s_tab[(x >> 8) & 255u].x << 8) | (s_tab[(x >> 16) & 255u].x << 16) |
                                (s_tab[x >> 24].x << 24);
                    }
                    st_nt(reinterpret_cast<uint4 *>(ob + blk_start + (uint64_t)k * PACK_TILE + (uint64_t)t * 16),
                          make_uint4(w4[0], w4[1], w4[2], w4[3]));
                }
            } else {
                for (uint64_t i = blk_start + t; i < blk_end; i += 256) ob[i] = (uint8_t)s_tab[in[i]].x;
            }
            // the stream's last word: its bytes past the stream are zero (the pad), whatever
            // the buffer held
            if (blk_end == n && t < 4 && ((n + 3) & ~3ull) > n + (uint64_t)t) ob[n + t] = 0;
            if (sync_len != nullptr) {   // chunks of S symbols: 8 S bits (the last: 8 x its symbols)
                for (uint64_t c = (blk_start >> slog) + t; c < ((blk_end + sync_syms - 1) >> slog); c += 256) {
                    const uint64_t s0 = c << slog;
                    sync_len[c] = (uint16_t)(8u * (uint32_t)min((uint64_t)sync_syms, n - s0));
                    if ((c & (DC_SYNC_GROUP - 1)) == 0) sync_base[c >> DC_SYNC_GROUP_LOG] = bit_base + 8 * s0;
                }
            }
        }
        return;
    }

    // two blocks per workgroup, grid-stride (r1, 1 GiB C2: 16384 workgroups 0.452 ms against
    // 0.481 at 4096, 0.469 at 32768, 0.504 at 1024)
    uint4 blkv[PACK_PIECES];
    auto load_block = [&](uint64_t bb) {
#pragma unroll
        for (int k = 0; k < (int)(DC_BLOCK_BYTES / PACK_TILE); ++k)
            blkv[k] = LD_PACK(reinterpret_cast<const uint4 *>(in + bb * (uint64_t)DC_BLOCK_BYTES + (uint64_t)k * PACK_TILE + (uint64_t)t * 16));
    };
    const uint64_t nfull = n / DC_BLOCK_BYTES;
    if (PF && bx < nfull) load_block(bx);
    for (uint64_t b = bx; b < nblocks; b += gstride) {
        const uint64_t blk_start = b * (uint64_t)DC_BLOCK_BYTES;
        const uint64_t blk_end = (blk_start + DC_BLOCK_BYTES < n) ? blk_start + DC_BLOCK_BYTES : n;
        const bool full = (blk_start + DC_BLOCK_BYTES <= n);
        const uint64_t bnext = b + gstride;   // (PF: its loads go out as pass B frees each piece)
        if (!PF && full) {
            // the whole 32 KiB block: 8 independent 16-B loads per lane in flight at once
            // (loading the next block ahead measured slower every way tried: in extra
            // registers -8% (147 VGPRs), into these registers once pass B is done -4%, into
            // the caches -10%)
#pragma unroll
            for (int k = 0; k < (int)(DC_BLOCK_BYTES / PACK_TILE); ++k)
                blkv[k] = LD_PACK(reinterpret_cast<const uint4 *>(in + blk_start + (uint64_t)k * PACK_TILE + (uint64_t)t * 16));
        }
        const uint64_t s_excl = block_off[b], s_bits = block_off[b + 1] - s_excl;
        const uint64_t blk_abs = bit_base + s_excl;
        const uint64_t blk_first_word = blk_abs >> 5;
        uint64_t tile_abs = blk_abs;
        const uint32_t nw_blk = (uint32_t)(((blk_abs & 31) + s_bits + 31) >> 5);
        // stage origin: the block's first word rounded down to a 16-B boundary of `out`, so
        // the store phase moves whole uint4s (sh = stage index of the block's first word)
        const uint32_t sh = vec_out ? (uint32_t)((blk_first_word - word_base) & 3) : 0u;
        if (full && nw_blk + sh <= PACK_BLK_WORDS) {
            // ---- fast path: the whole block at once, 3 barriers ----
            // lane t of wave w codes piece k = bytes [k*4096 + t*16, +16) of the block, as
            // two halves of 8 codes, each gathered into a 64-bit register (no per-code
            // flush) and OR-ed into the stage as at most 3 words. A half of more than 64
            // bits takes the per-code flush loop instead (exact, rare on text).
            const int lane = t & 63, wid = t >> 6;
            const uint32_t nwa = sh + nw_blk;
            uint32_t Tk[PACK_PIECES], Hk[PACK_PIECES], Ik[PACK_PIECES];
#pragma unroll
            for (int k = 0; k < PACK_PIECES; ++k) {
                const uint32_t w4[4] = {blkv[k].x, blkv[k].y, blkv[k].z, blkv[k].w};
                uint32_t s0 = 0, s1 = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i) s0 += s_nb8[(w4[i >> 2] >> (8 * (i & 3))) & 255u];
#pragma unroll
                for (int i = 8; i < 16; ++i) s1 += s_nb8[(w4[i >> 2] >> (8 * (i & 3))) & 255u];
                Hk[k] = s0;
                Tk[k] = s0 + s1;
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int k = 0; k < PACK_PIECES; ++k) Ik[k] = wave_scan_incl(Tk[k]);
            if (lane == 63) {
#pragma unroll
                for (int k = 0; k < PACK_PIECES; ++k) s_tot[k][wid] = Ik[k];
            }
            lds_barrier();
            const uint64_t org = (blk_first_word - sh) << 5;   // absolute bit of stage bit 0
            const uint32_t cm = sync_syms >> 4;                 // lanes per sync chunk
            uint64_t run = blk_abs;   // absolute bit where piece k starts
#pragma unroll
            for (int k = 0; k < PACK_PIECES; ++k) {
                uint32_t wo = 0, kt = 0;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    const uint32_t v = s_tot[k][w];
                    wo += (w < wid) ? v : 0u;
                    kt += v;
                }
                const uint64_t As = run + wo + (Ik[k] - Tk[k]);
                run += kt;
                const uint64_t p = blk_start + (uint64_t)k * PACK_TILE + (uint64_t)t * 16;
                if (sync_len != nullptr) {
                    // chunk bits = inclusive scan at the chunk's last lane - exclusive at its first
                    const uint32_t last = (cm == 4) ? (uint32_t)__builtin_amdgcn_update_dpp(0, (int)Ik[k], 0xff, 0xf, 0xf, false)
                                                    : (uint32_t)__shfl((int)Ik[k], lane | (int)(cm - 1), 64);
                    if ((p & (uint64_t)(sync_syms - 1)) == 0) {
                        sync_len[p >> slog] = (uint16_t)(last - (Ik[k] - Tk[k]));
                        if ((p & ((uint64_t)sync_syms * DC_SYNC_GROUP - 1)) == 0)
                            sync_base[p >> (slog + DC_SYNC_GROUP_LOG)] = As;
                    }
                }
                uint32_t w4[4] = {blkv[k].x, blkv[k].y, blkv[k].z, blkv[k].w};
                // opaque copy: stops the compiler from keeping pass A's lookup addresses live
                asm volatile("" : "+v"(w4[0]), "+v"(w4[1]), "+v"(w4[2]), "+v"(w4[3]));
                const uint32_t rel = (uint32_t)(As - org);
                // OR a right-justified run of nb <= 64 bits into the stage at bit pos (<= 3 words)
                // Branch-free: the run left-justified in 64 bits has zeros below it, so the
                // words it does not reach receive 0 (a no-op OR; some lane of a wave needs each
                // of the 3 ORs anyway, so skipping them per lane saved no LDS cycle and cost
                // compares and exec-mask branches). nb == 0 only for an all-zero acc (absent
                // symbols have code 0), where the unmasked shift by 64 & 63 = 0 is harmless.
                auto emit = [&](uint64_t acc, uint32_t nb, uint32_t pos) {
                    const uint64_t al = acc << ((64u - nb) & 63u);
                    const uint32_t hi = (uint32_t)(al >> 32), lo = (uint32_t)al, r = pos & 31u, wi = pos >> 5;
                    atomicOr(&s_stage[wi], hi >> r);
                    atomicOr(&s_stage[wi + 1], __builtin_amdgcn_alignbit(hi, lo, r));
                    atomicOr(&s_stage[wi + 2], __builtin_amdgcn_alignbit(lo, 0u, r));
                };
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint32_t Th = h ? Tk[k] - Hk[k] : Hk[k];
                    const uint32_t pos = h ? rel + Hk[k] : rel;
                    if (!qmode && Th <= 64u) {
                        // (a packed 32-bit code|length table measured 4% slower: the
                        // extraction VALU costs more than the uint2 reads' bank conflicts)
                        uint64_t acc = 0;
#pragma unroll
                        for (int i = 8 * h; i < 8 * h + 8; ++i) {
                            const uint2 e = s_tab[(w4[i >> 2] >> (8 * (i & 3))) & 255u];
                            acc = (acc << e.y) | e.x;
                        }
                        emit(acc, Th, pos);
                    } else {
                        // a half of more than 64 bits (skewed or long codes, e.g. C4's Zipf
                        // bytes), or every half in quarter mode: two quarters of 4 codes, each
                        // <= 64 bits unless codes exceed 16 bits, then code by code
                        uint32_t p = pos;
#pragma unroll
                        for (int qq = 0; qq < 2; ++qq) {
                            uint2 e[4];
                            uint32_t nq = 0;
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const int bi = 8 * h + 4 * qq + i;
                                const uint32_t wv = qq ? w4[2 * h + 1] : w4[2 * h];
                                e[i] = s_tab[(wv >> (8 * (bi & 3))) & 255u];
                                nq += e[i].y;
                            }
                            if (nq <= 64u) {
                                uint64_t acc = 0;
#pragma unroll
                                for (int i = 0; i < 4; ++i) acc = (acc << e[i].y) | e[i].x;
                                emit(acc, nq, p);
                                p += nq;
                            } else {
#pragma unroll
                                for (int i = 0; i < 4; ++i) { emit(e[i].x, e[i].y, p); p += e[i].y; }
                            }
                        }
                    }
                }
                if (PF && bnext < nfull)   // piece k of the next block, in flight through the rest
                    blkv[k] = LD_PACK(reinterpret_cast<const uint4 *>(in + bnext * (uint64_t)DC_BLOCK_BYTES + (uint64_t)k * PACK_TILE + (uint64_t)t * 16));
                __builtin_amdgcn_sched_barrier(0);   // keep the pieces' lookups from being hoisted
            }
            lds_barrier();
            // stage word sh = the block's first word, shared with the previous block; the last
            // word is shared with the next one when the block ends inside it: those two are
            // OR-ed into HBM by one lane each, the rest are plain stores (uint4 where whole)
            const uint32_t last_plain = ((run & 31) != 0) ? nwa - 1 : nwa;   // plain: [sh+1, last_plain)
            uint32_t *dst = out + (blk_first_word - word_base) - sh;
            // every stage word read below is zeroed by the thread that read it (the stage is
            // zero at the next block's start; words < sh and past nwa were never written)
            if (vec_out) {
                const uint32_t nq = last_plain >> 2;   // uint4 q covers stage words [4q, 4q+4)
                for (uint32_t q = 1 + t; q < nq; q += 256) {
                    uint4 *const sq = reinterpret_cast<uint4 *>(&s_stage[4 * q]);
                    const uint4 v = *sq;
                    *sq = make_uint4(0u, 0u, 0u, 0u);
                    // streaming (nt) stores: same-box A/B on 1 GiB C2, pack 0.420 -> 0.382 ms
                    // (the decode after it reads the payload no slower)
                    uint4 *const d4 = reinterpret_cast<uint4 *>(dst + 4 * q);
                    __builtin_nontemporal_store(bswap32(v.x), &d4->x);
                    __builtin_nontemporal_store(bswap32(v.y), &d4->y);
                    __builtin_nontemporal_store(bswap32(v.z), &d4->z);
                    __builtin_nontemporal_store(bswap32(v.w), &d4->w);
                }
                // head: words sh+1..3 of uint4 0; tail: words of the last, partial uint4
                const uint32_t hend = last_plain < 4u ? last_plain : 4u;
                if (t < 4 && (uint32_t)t > sh && (uint32_t)t < hend) { dst[t] = bswap32(s_stage[t]); s_stage[t] = 0u; }
                const uint32_t tb = nq > 0 ? 4 * nq : 4u;
                if (t >= 8 && t < 12 && tb + (t - 8) < last_plain) {
                    dst[tb + (t - 8)] = bswap32(s_stage[tb + (t - 8)]);
                    s_stage[tb + (t - 8)] = 0u;
                }
            } else {
                for (uint32_t i = t + 1; i < last_plain; i += 256) { dst[i] = bswap32(s_stage[i]); s_stage[i] = 0u; }
            }
            // the first word (shared with the previous block when the block starts inside it)
            // and the last (shared with the next one when the block ends inside it) are
            // OR-ed into HBM, where k_block_final_wide zeroed them (no-return atomics)
            if (t == 0) {
                atomicOr(&dst[sh], bswap32(s_stage[sh]));
                s_stage[sh] = 0u;
            }
            if (t == 64 && last_plain < nwa && nw_blk > 1) {
                atomicOr(&dst[nwa - 1], bswap32(s_stage[nwa - 1]));
                s_stage[nwa - 1] = 0u;
            }
            lds_barrier();
            continue;
        }
#pragma unroll
        for (int k = 0; k < (int)(DC_BLOCK_BYTES / PACK_TILE); ++k) {
            const uint64_t tile = blk_start + (uint64_t)k * PACK_TILE;
            if (tile >= blk_end) break;
            const uint64_t p = tile + (uint64_t)t * 16;
            const int cnt = (p + 16 <= blk_end) ? 16 : (p < blk_end ? (int)(blk_end - p) : 0);
            uint32_t bytes4[4] = {0u, 0u, 0u, 0u};
            if (full) {
                bytes4[0] = blkv[k].x; bytes4[1] = blkv[k].y; bytes4[2] = blkv[k].z; bytes4[3] = blkv[k].w;
            } else {
                for (int i = 0; i < cnt; ++i) bytes4[i >> 2] |= (uint32_t)in[p + i] << (8 * (i & 3));
            }
            uint32_t code[16], nb[16];
            uint32_t T_bits = 0;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint2 e = s_tab[(bytes4[i >> 2] >> (8 * (i & 3))) & 255u];
                code[i] = e.x;
                nb[i] = (i < cnt) ? e.y : 0u;
                T_bits += nb[i];
            }
            uint32_t tile_bits;
            const uint32_t pre = wg_scan_excl_u32(T_bits, s_scan, &tile_bits);
            const uint64_t TB = tile_abs >> 5;
            const uint64_t As = tile_abs + pre;
            const uint64_t Ae = As + T_bits;
            if (sync_len != nullptr) {
                // chunk = sync_syms symbols = sync_syms/16 consecutive lanes of one wave
                uint32_t cb = T_bits;
                for (uint32_t d = 1; d < (sync_syms >> 4); d <<= 1) cb += __shfl_xor(cb, (int)d, 64);
                if (cnt > 0 && (p & (uint64_t)(sync_syms - 1)) == 0) {
                    sync_len[p >> slog] = (uint16_t)cb;
                    if ((p & ((uint64_t)sync_syms * DC_SYNC_GROUP - 1)) == 0)
                        sync_base[p >> (slog + DC_SYNC_GROUP_LOG)] = As;
                }
            }
            const uint32_t ws = (uint32_t)((As >> 5) - TB);
            if (ws != 0) s_stage[ws] = 0u;
            if (t == 255) {
                const uint32_t we = (uint32_t)((Ae >> 5) - TB);
                if (we != 0) s_stage[we] = 0u;
            }
            __syncthreads();
            if (T_bits > 0) {
                uint64_t acc = 0;
                uint32_t nacc = (uint32_t)(As & 31);
                uint32_t wi = ws;
                bool first = true;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    if (nb[i]) {
                        acc = (acc << nb[i]) | code[i];
                        nacc += nb[i];
                        if (nacc >= 32) {
                            nacc -= 32;
                            const uint32_t word = (uint32_t)(acc >> nacc);
                            if (first) atomicOr(&s_stage[wi], word);
                            else s_stage[wi] = word;
                            first = false;
                            ++wi;
                        }
                    }
                }
                if (nacc > 0) atomicOr(&s_stage[wi], (uint32_t)(acc << (32 - nacc)));
            }
            __syncthreads();
            const uint64_t tile_end_abs = tile_abs + tile_bits;
            const uint32_t nfull = (uint32_t)((tile_end_abs >> 5) - TB);
            for (uint32_t i = t; i < nfull; i += 256) {
                const uint64_t gw = TB + i;
                if (gw == blk_first_word) atomicOr(&out[gw - word_base], bswap32(s_stage[i]));
                else out[gw - word_base] = bswap32(s_stage[i]);
            }
            __syncthreads();
            if (t == 0) s_stage[0] = (tile_end_abs & 31) ? s_stage[nfull] : 0u;
            tile_abs = tile_end_abs;
            __syncthreads();
        }
        if (t == 0 && (tile_abs & 31)) atomicOr(&out[(tile_abs >> 5) - word_base], bswap32(s_stage[0]));   // partial last word
        __syncthreads();
        // the tile loop leaves its stage dirty: zero it for the next block (rare path)
        for (uint32_t i = 4u * t; i < PACK_BLK_WORDS + 4; i += 1024u)
            *reinterpret_cast<uint4 *>(&s_stage[i]) = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
        if (PF && bnext < nfull) load_block(bnext);
    }
}

// C5 fused front-end pack: codes the front-end output M of `in` (see the front-end fusion
// block above k_hist_blocks) without M ever being written. The blocks are k_huff_pack's: 32 KiB
// of the INPUT, lane t of wave w coding piece k = input bytes [k*4096 + 16t, +16), whose
// symbols are the bytes y: x, or letter | 0x80 at a pair's second position, or z (a byte value
// without a code: 0 bits) at a pair's start and past the input. Block b's bit offset comes
// from the plan over the FE histograms, its first symbol index msym[b] from the same plan.
// The sync index (chunks of S symbols of M) is k_huff_pack's format, but chunk starts no longer
// sit at piece starts: a lane whose piece holds the symbol of index = 0 mod S (at most one:
// S >= 16) records that symbol's bit offset (bits of the piece before it, tallied in pass B)
// in a list beside the stage; after pass B the block writes each chunk's length as the
// difference of consecutive starts. The chunks spanning a block boundary get their two parts
// by atomic adds into the u32 holding their u16 (zeroed by the plan), and so does the other
// u16 of that u32. Fallbacks (reported in the plan slot's err[1], nothing written): LITERAL
// output (M >= n bytes), no free byte value for z, a block whose bits exceed the stage.
// SH (a shard of the stream, dist.ShardedSmall at world > 1; shard = FeShard): the shard's
// context bytes (fe_ctx), its codes at the global bit shard[0] (the words start at global word
// shard[0] / 32), its local sync index (chunks from its own first symbol: its own decode), and
// the stream's GLOBAL sync index over its symbols, chunks at multiples of S of the global symbol
// index shard[1]: gsync_len (u16, entry c - (c0 & ~1) for global chunk c, c0 = the shard's first;
// the first and last chunks hold this shard's part only, the gather adds the neighbours') and
// gsync_base (group g at entry g - ceil(shard[1] / 64 S): the groups that start in this shard).
// Bits of a piece before its symbol number jj (and jjg): the sum of the lengths L (a byte per
// position, 0 = no symbol) of the positions whose inclusive symbol count is <= jj. Counts by
// SWAR prefix sums per dword, the sums by v_dot4 against the 0/1 bytes of the compare.
template <bool SH>
static __device__ __forceinline__ void fe_chunk_bits(const uint32_t (&L)[4], uint32_t jj, uint32_t jjg, uint32_t &cap,
                                                     uint32_t &capg)
{
    const uint32_t J = 0x80808080u + min(jj, 16u) * 0x01010101u, Jg = 0x80808080u + min(jjg, 16u) * 0x01010101u;
    uint32_t prev = 0;   // the symbol count before the dword, in every byte
    cap = 0;
    capg = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t nz = ((L[q] + 0x7F7F7F7Fu) >> 7) & 0x01010101u;   // 1 per position with a symbol
        const uint32_t y = nz + (nz << 8);
        const uint32_t C = y + (y << 16) + prev;                          // inclusive counts (<= 16)
        prev = __builtin_amdgcn_perm(0u, C, 0x03030303u);
        cap = __builtin_amdgcn_udot4(L[q], ((J - C) >> 7) & 0x01010101u, cap, false);
        if (SH) capg = __builtin_amdgcn_udot4(L[q], ((Jg - C) >> 7) & 0x01010101u, capg, false);
    }
}

template <bool SH>
__global__ __launch_bounds__(256) void k_fe_pack(const uint8_t *__restrict__ in, uint64_t n,
                                                 const dc_dtable *__restrict__ T,
                                                 const uint64_t *__restrict__ block_off,
                                                 const uint64_t *__restrict__ msym, uint64_t bit_base,
                                                 uint32_t *__restrict__ out, uint64_t *__restrict__ sync_base,
                                                 uint16_t *__restrict__ sync_len, uint32_t sync_syms,
                                                 uint64_t nblocks, uint64_t words_cap, int *__restrict__ err,
                                                 int build_dec, const int64_t *__restrict__ shard = nullptr,
                                                 uint64_t *__restrict__ gsync_base = nullptr,
                                                 uint16_t *__restrict__ gsync_len = nullptr)
{
    __shared__ uint2 s_tab[256];
    __shared__ uint8_t s_nb8[256];
    __shared__ __attribute__((aligned(16))) uint32_t s_stage[PACK_BLK_WORDS + 4];
    __shared__ uint32_t s_tot[PACK_PIECES][4];
    __shared__ uint32_t s_z;
    static_assert(sizeof(DecBuildLds) <= sizeof(s_stage), "decoder-table builder uses the stage");
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    if (build_dec && blockIdx.x == 0) {
        if (T->status == DC_OK)
            dec_tables_build(const_cast<dc_dtable *>(T), *reinterpret_cast<DecBuildLds *>(s_stage));
        return;
    }
    const uint64_t bx = blockIdx.x - (uint64_t)build_dec, gstride = gridDim.x - (uint64_t)build_dec;
    const uint64_t total = block_off[nblocks];
    const FeCtx fc = fe_ctx(SH ? shard : nullptr);
    const uint64_t M = SH ? (uint64_t)shard[1] : 0;   // the shard's first symbol, global index
    if (SH) bit_base += (uint64_t)shard[0];
    if (err[0] != 0) return;
    if (((bit_base & 31) + total + 31) / 32 > words_cap) {
        if (t == 0) err[2] = 1;
        return;
    }
    const uint32_t nbt = T->nbits[t];
    s_tab[t] = make_uint2(nbt ? T->code[t] : 0u, nbt);   // z codes as nothing (a code value of a
    s_nb8[t] = (uint8_t)nbt;                               // length-0 entry would be OR-ed in)
    if (t == 0) s_z = 256u;
    for (uint32_t i = 4u * t; i < PACK_BLK_WORDS + 4; i += 1024u)
        *reinterpret_cast<uint4 *>(&s_stage[i]) = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    const uint64_t zb = __ballot(nbt == 0u);   // byte values without a code
    if (lane == 0 && zb) atomicMin(&s_z, (uint32_t)(t + __builtin_ctzll(zb)));
    __syncthreads();
    const uint32_t z = s_z;
    const uint64_t mtot = msym[nblocks];   // symbols of M (the type byte included)
    if (z > 255u || (!SH && mtot >= n)) {   // (a shard: the LITERAL test is the whole stream's)
        if (t == 0) err[1] = 1;
        return;
    }
    const bool vec_out = ((uintptr_t)out & 15) == 0;
    const uint64_t word_base = bit_base >> 5;
    const uint32_t slog = (uint32_t)__builtin_ctz(sync_syms), S = sync_syms;
    const uint32_t cbw = (DC_BLOCK_BYTES >> slog) + 2;             // chunk starts a block can hold
    uint32_t *const s_cb = s_stage + (PACK_BLK_WORDS + 4 - cbw);   // the list sits past the payload
    uint32_t *const s_cbg = s_cb - (SH ? cbw : 0u);                 // SH: the global chunks' starts
    const uint32_t lim = PACK_BLK_WORDS - (SH ? 2 : 1) * cbw - 4;
    const uint64_t c0e = SH ? (M >> slog) & ~1ull : 0;                  // global chunk of gsync_len[0]
    const uint64_t g0 = SH ? (M + ((uint64_t)S << DC_SYNC_GROUP_LOG) - 1) >> (slog + DC_SYNC_GROUP_LOG) : 0;
    uint32_t *const gl32 = reinterpret_cast<uint32_t *>(gsync_len);
    const bool qmode = 2 * total > 11 * mtot;
    const uint32_t Z4 = z * 0x01010101u;
    uint32_t *const sl32 = reinterpret_cast<uint32_t *>(sync_len);

    for (uint64_t b = bx; b < nblocks; b += gstride) {
        const uint64_t blk_start = b * (uint64_t)DC_BLOCK_BYTES;
        const bool full = blk_start + DC_BLOCK_BYTES <= n;
        uint4 blkv[PACK_PIECES];
        uint32_t ve[PACK_PIECES];
        if (full) {
#pragma unroll
            for (int k = 0; k < PACK_PIECES; ++k) {
                const uint64_t p = blk_start + (uint64_t)k * PACK_TILE + (uint64_t)t * 16;
                blkv[k] = LD_PACK(reinterpret_cast<const uint4 *>(in + p));
                ve[k] = *reinterpret_cast<const uint32_t *>(in + fe_edge_addr(p, lane, n));
            }
        } else {   // the stream's last, partial block: bytes past the input read as 0 (the 16-B
                   // granule holding byte n - 1 is read whole: it lies in the page of that byte)
#pragma unroll
            for (int k = 0; k < PACK_PIECES; ++k) {
                const uint64_t p = blk_start + (uint64_t)k * PACK_TILE + (uint64_t)t * 16;
                uint4 v = p < n ? LD_PACK(reinterpret_cast<const uint4 *>(in + p)) : make_uint4(0u, 0u, 0u, 0u);
                if (p + 16 > n) {
                    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int64_t r = (int64_t)n - (int64_t)(p + 4 * q);   // bytes of dword q inside
                        w[q] &= r <= 0 ? 0u : r >= 4 ? ~0u : ~(~0u << (8 * (uint32_t)r));
                    }
                    v = make_uint4(w[0], w[1], w[2], w[3]);
                }
                if (SH && n >= p && n < p + 16) {   // the byte after the shard (pair starts at n - 1)
                    uint32_t w[4] = {v.x, v.y, v.z, v.w};
                    const uint32_t o = (uint32_t)(n - p);
#pragma unroll
                    for (int q = 0; q < 4; ++q) w[q] |= (uint32_t)q == (o >> 2) ? fc.rb << (8 * (o & 3)) : 0u;
                    v = make_uint4(w[0], w[1], w[2], w[3]);
                }
                blkv[k] = v;
                const uint64_t ea = fe_edge_addr(p, lane, n);
                ve[k] = ea < n ? *reinterpret_cast<const uint32_t *>(in + ea) : 0u;
            }
        }
        const uint64_t s_excl = block_off[b], s_bits = block_off[b + 1] - s_excl;
        const uint64_t blk_abs = bit_base + s_excl;
        const uint64_t blk_first_word = blk_abs >> 5;
        const uint32_t nw_blk = (uint32_t)(((blk_abs & 31) + s_bits + 31) >> 5);
        const uint32_t sh = vec_out ? (uint32_t)((blk_first_word - word_base) & 3) : 0u;
        if (nw_blk + sh > lim) {   // uniform: more bits than the stage holds beside the list
            if (t == 0) err[1] = 2;
            continue;
        }
        const uint64_t m0 = msym[b], m1 = msym[b + 1];
        const uint64_t cf = (m0 + S - 1) >> slog;   // the first chunk that starts in this block
        const uint64_t ct = (m1 - 1) >> slog;       // the last one (this block's tail chunk)
        const uint32_t nc = ct >= cf ? (uint32_t)(ct - cf + 1) : 0u;
        const uint64_t cfg = (M + m0 + S - 1) >> slog, ctg = (M + m1 - 1) >> slog;   // (SH: global chunks)
        const uint32_t ncg = SH && ctg >= cfg ? (uint32_t)(ctg - cfg + 1) : 0u;
        const uint32_t nwa = sh + nw_blk;
        // ---- the symbols y, pass A: bit and symbol counts per piece ----
        // Pk = bits (<= 512) | symbols << 18 (<= 16) | bits of the first half << 23 (<= 256)
        uint32_t Pk[PACK_PIECES], Ik[PACK_PIECES];
#pragma unroll
        for (int k = 0; k < PACK_PIECES; ++k) {
            const uint64_t p = blk_start + (uint64_t)k * PACK_TILE + (uint64_t)t * 16;
            uint32_t w4[4] = {blkv[k].x, blkv[k].y, blkv[k].z, blkv[k].w};
            const uint32_t pd = dpp_wave_shr1(w4[3]), qd = dpp_wave_shl1(w4[0]);   // (statements of their own)
            const uint32_t pb = lane == 0 ? (p == 0 ? fc.lb : ve[k] >> 24) : pd >> 24;
            const uint32_t qb = lane == 63 ? (p + 16 < n ? ve[k] & 255u : fc.rb) : qd & 255u;
            uint32_t st[4];
            fe_pair_starts(w4, qb, st);
            if (p == 0 && fc.first) st[0] &= ~0x80u;   // the stream's position 0 never starts a pair
            uint32_t nul = 0;               // positions without a symbol
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t sec = (st[q] << 8) | (q ? st[q - 1] >> 24 : fe_start_before(pb, w4[0], fc.first ? p : 16));
                uint32_t m8 = st[q];
                if (!full) {   // past the input: no symbol
                    const int64_t v = (int64_t)n - (int64_t)(p + 4 * q);
                    m8 |= v <= 0 ? 0x80808080u : v >= 4 ? 0u : (0x80808080u << (8 * (uint32_t)v));
                }
                nul += (uint32_t)__popc(m8);
                m8 = (m8 - (m8 >> 7)) | m8;   // 0x80 -> 0xFF per byte
                w4[q] = (w4[q] & ~m8) | (Z4 & m8) | sec;
            }
            blkv[k] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
            uint32_t s0 = 0, s1 = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) s0 += s_nb8[(w4[i >> 2] >> (8 * (i & 3))) & 255u];
#pragma unroll
            for (int i = 8; i < 16; ++i) s1 += s_nb8[(w4[i >> 2] >> (8 * (i & 3))) & 255u];
            Pk[k] = (s0 + s1) | ((16u - nul) << 18) | (s0 << 23);
            // materialised here: sunk to the scan, the sums kept every piece's 16 lookups live
            asm volatile("" : "+v"(Pk[k]));
            __builtin_amdgcn_sched_barrier(0);
        }
        // one scan of bits | symbols << 18 (a piece of the workgroup: <= 2^17 bits, 4096 symbols)
#pragma unroll
        for (int k = 0; k < PACK_PIECES; ++k) Ik[k] = wave_scan_incl(Pk[k] & 0x7FFFFFu);
        if (lane == 63) {
#pragma unroll
            for (int k = 0; k < PACK_PIECES; ++k) s_tot[k][wid] = Ik[k];
        }
        lds_barrier();
        const uint64_t org = (blk_first_word - sh) << 5;   // absolute bit of stage bit 0
        auto emit = [&](uint64_t acc, uint32_t nb, uint32_t pos) {   // as in k_huff_pack
            const uint64_t al = acc << ((64u - nb) & 63u);
            const uint32_t hi = (uint32_t)(al >> 32), lo = (uint32_t)al, r = pos & 31u, wi = pos >> 5;
            atomicOr(&s_stage[wi], hi >> r);
            atomicOr(&s_stage[wi + 1], __builtin_amdgcn_alignbit(hi, lo, r));
            atomicOr(&s_stage[wi + 2], __builtin_amdgcn_alignbit(lo, 0u, r));
        };
        uint64_t run = blk_abs, mrun = m0;
        if (b == 0 && fc.first) {   // M[0] = the type byte 8 (EIGHT_BIT_PRUNED, small_compression.c:39), chunk 0's start
            const uint2 h = s_tab[8];
            if (t == 0) {
                emit(h.x, h.y, (uint32_t)(blk_abs - org));
                s_cb[0] = 0u;
                if (SH) s_cbg[0] = 0u;   // (the first shard: global = local)
            }
            run += h.y;
            mrun += 1;
        }
#pragma unroll
        for (int k = 0; k < PACK_PIECES; ++k) {
            uint32_t wo = 0, kt = 0, cwo = 0, ckt = 0;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const uint32_t v = s_tot[k][w], vb = v & 0x3FFFFu, vc = v >> 18;
                wo += (w < wid) ? vb : 0u;
                kt += vb;
                cwo += (w < wid) ? vc : 0u;
                ckt += vc;
            }
            const uint32_t Tk = Pk[k] & 0x3FFFFu, Ck = (Pk[k] >> 18) & 31u, Hk = Pk[k] >> 23;
            const uint64_t As = run + wo + ((Ik[k] & 0x3FFFFu) - Tk);
            const uint64_t mi = mrun + cwo + ((Ik[k] >> 18) - Ck);   // index of the piece's first symbol
            run += kt;
            mrun += ckt;
            const uint32_t j0 = (uint32_t)(0ull - mi) & (S - 1);     // symbols before the chunk start
            const bool has = j0 < Ck;
            const uint32_t jj = has ? j0 : 0xFFFFu;
            const uint32_t j0g = (uint32_t)(0ull - (mi + M)) & (S - 1);   // (SH: the global chunk start)
            const bool hasg = SH && j0g < Ck;
            const uint32_t jjg = hasg ? j0g : 0xFFFFu;
            // the piece's code lengths, a byte each (<= 32), for the chunk start's bit offset
            // after pass B (fe_chunk_bits: SWAR, ~3.75 VALU per symbol with the packing; the
            // per-symbol count and compare it replaced cost ~5: fe_pack 0.671 -> 0.641 ms per GiB
            // of C5, profiles/r6k_fe_tally_nyb_ranks_ab.log)
            uint32_t L4[4] = {0u, 0u, 0u, 0u};
            auto tally = [&](int i, uint32_t l) {
                L4[i >> 2] = (i & 3) ? L4[i >> 2] | (l << (8 * (i & 3))) : l;
            };
            uint32_t w4[4] = {blkv[k].x, blkv[k].y, blkv[k].z, blkv[k].w};
            asm volatile("" : "+v"(w4[0]), "+v"(w4[1]), "+v"(w4[2]), "+v"(w4[3]));
            const uint32_t rel = (uint32_t)(As - org);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t Th = h ? Tk - Hk : Hk;
                const uint32_t pos = h ? rel + Hk : rel;
                if (!qmode && Th <= 64u) {
                    uint64_t acc = 0;
#pragma unroll
                    for (int i = 8 * h; i < 8 * h + 8; ++i) {
                        const uint2 e = s_tab[(w4[i >> 2] >> (8 * (i & 3))) & 255u];
                        acc = (acc << e.y) | e.x;
                        tally(i, e.y);
                    }
                    emit(acc, Th, pos);
                } else {
                    uint32_t pq = pos;
#pragma unroll
                    for (int qq = 0; qq < 2; ++qq) {
                        uint2 e[4];
                        uint32_t nq = 0;
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int bi = 8 * h + 4 * qq + i;
                            const uint32_t wv = qq ? w4[2 * h + 1] : w4[2 * h];
                            e[i] = s_tab[(wv >> (8 * (bi & 3))) & 255u];
                            nq += e[i].y;
                            tally(bi, e[i].y);
                        }
                        if (nq <= 64u) {
                            uint64_t acc = 0;
#pragma unroll
                            for (int i = 0; i < 4; ++i) acc = (acc << e[i].y) | e[i].x;
                            emit(acc, nq, pq);
                            pq += nq;
                        } else {
#pragma unroll
                            for (int i = 0; i < 4; ++i) { emit(e[i].x, e[i].y, pq); pq += e[i].y; }
                        }
                    }
                }
            }
            uint32_t cap, capg = 0;   // bits before the chunk starts
            fe_chunk_bits<SH>(L4, jj, jjg, cap, capg);
            if (has) s_cb[(uint32_t)(((mi + j0) >> slog) - cf)] = (uint32_t)(As - blk_abs) + cap;
            if (hasg) s_cbg[(uint32_t)(((mi + M + j0g) >> slog) - cfg)] = (uint32_t)(As - blk_abs) + capg;
            __builtin_amdgcn_sched_barrier(0);
        }
        lds_barrier();
        // ---- store phase: as in k_huff_pack ----
        const uint32_t last_plain = ((run & 31) != 0) ? nwa - 1 : nwa;
        uint32_t *dst = out + (blk_first_word - word_base) - sh;
        if (vec_out) {
            const uint32_t nq = last_plain >> 2;
            for (uint32_t q = 1 + t; q < nq; q += 256) {
                uint4 *const sq = reinterpret_cast<uint4 *>(&s_stage[4 * q]);
                const uint4 v = *sq;
                *sq = make_uint4(0u, 0u, 0u, 0u);
                uint4 *const d4 = reinterpret_cast<uint4 *>(dst + 4 * q);
                __builtin_nontemporal_store(bswap32(v.x), &d4->x);
                __builtin_nontemporal_store(bswap32(v.y), &d4->y);
                __builtin_nontemporal_store(bswap32(v.z), &d4->z);
                __builtin_nontemporal_store(bswap32(v.w), &d4->w);
            }
            const uint32_t hend = last_plain < 4u ? last_plain : 4u;
            if (t < 4 && (uint32_t)t > sh && (uint32_t)t < hend) { dst[t] = bswap32(s_stage[t]); s_stage[t] = 0u; }
            const uint32_t tb = nq > 0 ? 4 * nq : 4u;
            if (t >= 8 && t < 12 && tb + (t - 8) < last_plain) {
                dst[tb + (t - 8)] = bswap32(s_stage[tb + (t - 8)]);
                s_stage[tb + (t - 8)] = 0u;
            }
        } else {
            for (uint32_t i = t + 1; i < last_plain; i += 256) { dst[i] = bswap32(s_stage[i]); s_stage[i] = 0u; }
        }
        if (t == 0) {
            atomicOr(&dst[sh], bswap32(s_stage[sh]));
            s_stage[sh] = 0u;
        }
        if (t == 64 && last_plain < nwa && nw_blk > 1) {
            atomicOr(&dst[nwa - 1], bswap32(s_stage[nwa - 1]));
            s_stage[nwa - 1] = 0u;
        }
        // ---- the sync index: chunk lengths from consecutive starts; group bases ----
        if (sync_len != nullptr) {
            const uint64_t hd = m0 > 0 ? ((m0 - 1) >> slog) >> 1 : ~0ull, td = ct >> 1;
            for (uint32_t i = t; i < nc; i += 256) {
                const uint32_t a = s_cb[i], e = i + 1 < nc ? s_cb[i + 1] : (uint32_t)s_bits;
                const uint64_t c = cf + i;
                if ((c & (DC_SYNC_GROUP - 1)) == 0) sync_base[c >> DC_SYNC_GROUP_LOG] = blk_abs + a;
                if ((c >> 1) == hd || (c >> 1) == td) atomicAdd(&sl32[c >> 1], (e - a) << (16u * (uint32_t)(c & 1)));
                else sync_len[c] = (uint16_t)(e - a);
            }
            if (t == 255 && (m0 & (S - 1)) != 0) {   // the previous block's tail chunk: the part in this block
                const uint64_t c = cf - 1;
                atomicAdd(&sl32[c >> 1], (nc ? s_cb[0] : (uint32_t)s_bits) << (16u * (uint32_t)(c & 1)));
            }
            if (SH) {   // the same over the global chunks (the shard's first and last chunks are partial)
                const uint64_t hdg = M + m0 > 0 ? ((M + m0 - 1) >> slog) >> 1 : ~0ull, tdg = ctg >> 1;
                for (uint32_t i = t; i < ncg; i += 256) {
                    const uint32_t a = s_cbg[i], e = i + 1 < ncg ? s_cbg[i + 1] : (uint32_t)s_bits;
                    const uint64_t c = cfg + i, ix = c - c0e;
                    if ((c & (DC_SYNC_GROUP - 1)) == 0) gsync_base[(c >> DC_SYNC_GROUP_LOG) - g0] = blk_abs + a;
                    if ((c >> 1) == hdg || (c >> 1) == tdg) atomicAdd(&gl32[ix >> 1], (e - a) << (16u * (uint32_t)(ix & 1)));
                    else gsync_len[ix] = (uint16_t)(e - a);
                }
                if (t == 254 && ((M + m0) & (S - 1)) != 0) {
                    const uint64_t c = cfg - 1, ix = c - c0e;
                    atomicAdd(&gl32[ix >> 1], (ncg ? s_cbg[0] : (uint32_t)s_bits) << (16u * (uint32_t)(ix & 1)));
                }
            }
        }
        lds_barrier();
    }
}

// ------------------------------------------------------------------------------------
// (H8) decode. The stream is cut into chunks of S symbols (sync index: u16 bit length per
// chunk, u64 absolute bit offset per group of 64 chunks). One wave decodes one group,
// one lane per chunk:
//  1. lanes read the 64 chunk lengths (one coalesced 128-B load) and prefix-sum them;
//  2. the wave copies the group's whole compressed span (contiguous) into its private LDS
//     staging area with 16-B loads, 1 KiB per wave-instruction, then waits once;
//  3. each lane decodes its chunk from LDS: 64-bit MSB-first window refilled from the
//     staged words, 12-bit first-level LDS table, canonical limit compare for longer
//     codes (n a power of two) or a base-n digit walk (other n);
//  4. 16 decoded bytes per lane -> one 16-B store.
// A group whose span exceeds the staging area is decoded straight from HBM (fallback).
// Persistent grid: each workgroup loads the tables once and walks groups grid-stride.
// ------------------------------------------------------------------------------------
#define DEC_WAVES 16            /* one 1024-thread workgroup per CU shares the 16 KiB table   */
#define DEC_STAGE_WORDS 1088   /* 4.25 KiB compressed input per wave                          */
#define DEC_OUT_SYMS 64        /* chunks of <= 64 symbols are staged through LDS for output   */
#define DEC_OUT_STRIDE 72      /* bytes per lane: 64 + 8 pad (overshoot room), 18-dword rows  */

// table entry (dc_gpu.h): sym0 | bits(all)<<8 | sym1<<16 | bits(sym0)<<24 | count<<29
#define E_BITS(e) (((e) >> 8) & 255u)
#define E_BITS0(e) (((e) >> 24) & 31u)
#define E_COUNT(e) (((e) >> 29) & 3u)

struct DecLds {
    uint32_t lut[1 << DC_LUT_BITS];   // first: its addresses fit the ds_read offset field
    uint32_t first[DC_MAX_DIGITS + 1], count[DC_MAX_DIGITS + 1], start[DC_MAX_DIGITS + 1];
    uint16_t syms[DC_MAX_SYMS];
    __attribute__((aligned(16))) uint32_t stage[DEC_WAVES][DEC_STAGE_WORDS];
    __attribute__((aligned(16))) uint8_t out[DEC_WAVES][64 * DEC_OUT_STRIDE];
};

// Word readers; nx = the next word to enter the window (already MSB-first), p = the one after.
struct LdsWords {   // staged words are byte-swapped once at staging time
    const uint32_t *p;
    uint32_t nx;
    __device__ __forceinline__ void init() { nx = *p++; }
    __device__ __forceinline__ uint32_t peek() const { return nx; }
    __device__ __forceinline__ void advance(bool take)   // LDS read every step, kept when taken
    {
        const uint32_t v = *p;
        nx = take ? v : nx;
        p += take ? 1 : 0;
    }
};

struct HbmWords {   // HBM fallback: byte-swap on read, read only when a word is taken
    const uint32_t *p;
    uint32_t nx;
    __device__ __forceinline__ void init() { nx = bswap32(*p++); }
    __device__ __forceinline__ uint32_t peek() const { return nx; }
    __device__ __forceinline__ void advance(bool take)
    {
        if (take) { nx = bswap32(*p); ++p; }
    }
};

// slow path for windows the two-symbol table does not cover (codes longer than 12 bits);
// returns a one-symbol table entry, bit 31 set for an invalid code
static __device__ __forceinline__ uint32_t decode_long(uint64_t win, const DecLds &L, const dc_dtable *__restrict__ T,
                                                       int nary, int w, bool pow2)
{
    uint32_t bad = 0, sym = 0, nbt;
    if (pow2) {
        // smallest bit length b > 12 whose left-justified canonical limit exceeds the window
        const uint64_t top = win >> 32;
        uint32_t b = DC_LUT_BITS + 1;
        for (int bb = DC_LUT_BITS + 1; bb <= 32; ++bb) b += (top >= T->lim[bb]) ? 1u : 0u;
        if (b > 32) { bad = 1; b = 32; }
        const uint32_t Ld = b / (uint32_t)w;
        const uint32_t v = (uint32_t)(top >> (32 - b));
        sym = L.syms[(L.start[Ld] + (v - L.first[Ld])) & (DC_MAX_SYMS - 1)];
        nbt = b;
    } else {
        uint64_t x = win;
        uint32_t v = 0;
        int Ld = 0;
        nbt = (uint32_t)w;
        while (true) {
            const uint32_t digit = (uint32_t)(x >> (64 - w));
            x <<= w;
            v = v * (uint32_t)nary + digit;
            ++Ld;
            if (Ld * w > 32 || Ld > DC_MAX_DIGITS) { bad = 1; break; }
            if (L.count[Ld] && v - L.first[Ld] < L.count[Ld]) {
                sym = L.syms[L.start[Ld] + (v - L.first[Ld])];
                nbt = (uint32_t)(Ld * w);
                break;
            }
        }
    }
    return (sym & 255u) | (nbt << 8) | (nbt << 24) | (1u << 29) | (bad << 31);
}

// One lookup step: refill (branch-free), table lookup, slow path for long codes.
template <class R>
static __device__ __forceinline__ uint32_t decode_step(R &rd, uint64_t &win, int &wbits, const DecLds &L,
                                                       const dc_dtable *__restrict__ T, int nary, int w, bool pow2,
                                                       int &bad)
{
    const bool need = wbits < 32;
    const uint64_t add = ((uint64_t)rd.peek() << 32) >> (need ? wbits : 0);
    win |= need ? add : 0ull;
    wbits += need ? 32 : 0;
    rd.advance(need);
    uint32_t e = L.lut[win >> (64 - DC_LUT_BITS)];
    if (__builtin_expect(__any(e == 0), 0)) {
        if (e == 0) {
            e = decode_long(win, L, T, nary, w, pow2);
            bad |= (int)(e >> 31);
        }
    }
    return e;
}

// decode into the lane's LDS row; the last step may write one byte past cnt (row padding)
template <class R>
static __device__ __forceinline__ void decode_chunk_lds(R rd, uint32_t sh, uint32_t cnt, uint8_t *row,
                                                        const DecLds &L, const dc_dtable *__restrict__ T, int nary,
                                                        int w, bool pow2, int &bad)
{
    rd.init();
    const uint32_t hi = rd.peek();
    rd.advance(true);
    const uint32_t lo = rd.peek();
    rd.advance(true);
    uint64_t win = (((uint64_t)hi << 32) | lo) << sh;
    int wbits = 64 - (int)sh;
    for (uint32_t pos = 0; pos < cnt;) {
        const uint32_t e = decode_step(rd, win, wbits, L, T, nary, w, pow2, bad);
        row[pos] = (uint8_t)e;
        row[pos + 1] = (uint8_t)(e >> 16);   // sym1, or a byte the next step overwrites
        const uint32_t nbt = E_BITS(e);
        win <<= nbt;
        wbits -= (int)nbt;
        pos += E_COUNT(e);
    }
}

// exact variant writing straight to HBM (chunks of more than 64 symbols)
template <class R>
static __device__ __forceinline__ void decode_chunk_hbm(R rd, uint32_t sh, uint32_t cnt, uint8_t *__restrict__ o,
                                                        const DecLds &L, const dc_dtable *__restrict__ T, int nary,
                                                        int w, bool pow2, int &bad)
{
    rd.init();
    const uint32_t hi = rd.peek();
    rd.advance(true);
    const uint32_t lo = rd.peek();
    rd.advance(true);
    uint64_t win = (((uint64_t)hi << 32) | lo) << sh;
    int wbits = 64 - (int)sh;
    for (uint32_t pos = 0; pos < cnt;) {
        const uint32_t e = decode_step(rd, win, wbits, L, T, nary, w, pow2, bad);
        const bool two = E_COUNT(e) == 2 && pos + 1 < cnt;
        o[pos] = (uint8_t)e;
        if (two) o[pos + 1] = (uint8_t)(e >> 16);
        const uint32_t nbt = two ? E_BITS(e) : E_BITS0(e);
        win <<= nbt;
        wbits -= (int)nbt;
        pos += two ? 2 : 1;
    }
}

__global__ __launch_bounds__(DEC_WAVES * 64) void k_huff_decode(const uint32_t *__restrict__ in, uint64_t bit_base, const uint64_t *__restrict__ d_base,
                                                     const uint64_t *__restrict__ sync_base,
                                                     const uint16_t *__restrict__ sync_len, uint32_t S,
                                                     uint64_t n, const dc_dtable *__restrict__ T,
                                                     uint8_t *__restrict__ out, int *__restrict__ err,
                                                     int *__restrict__ err_next)
{
    __shared__ DecLds L;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (blockIdx.x == 0 && t < 4) err_next[t] = 0;   // the next decode's error slot
    if (!__hip_atomic_load(&T->dec_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {   // tables rebuilt since
        if (threadIdx.x == 0) atomicOr(err, 1);
        return;
    }
    if (d_base) bit_base += *d_base;   // device-resident shard offset (dist: no host read)
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(T->lut);
        uint4 *dst = reinterpret_cast<uint4 *>(L.lut);
        for (int i = t; i < (1 << DC_LUT_BITS) / 4; i += DEC_WAVES * 64) dst[i] = src[i];
        for (int k = t; k <= DC_MAX_DIGITS; k += DEC_WAVES * 64) {
            L.first[k] = T->first[k]; L.count[k] = T->count[k]; L.start[k] = T->start[k];
        }
        for (int i = t; i < DC_MAX_SYMS; i += DEC_WAVES * 64) L.syms[i] = T->syms[i];
    }
    const int nary = T->n_ary, w = T->w;
    const bool pow2 = (nary & (nary - 1)) == 0;
    __syncthreads();

    const uint32_t slog = (uint32_t)__builtin_ctz(S);   // S is a power of two (checked by the host)
    const uint64_t nchunks = (n + S - 1) >> slog;
    const uint64_t ngroups = (nchunks + DC_SYNC_GROUP - 1) / DC_SYNC_GROUP;
    const uint64_t word_base = bit_base >> 5;
    uint32_t *stage = L.stage[wv];
    uint8_t *ostage = L.out[wv];
    const bool stage_out = S <= DEC_OUT_SYMS;
    int bad = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * DEC_WAVES + wv; g < ngroups; g += (uint64_t)gridDim.x * DEC_WAVES) {
        const uint64_t c = g * DC_SYNC_GROUP + lane;
        const bool valid = c < nchunks;
        const uint32_t len = valid ? sync_len[c] : 0u;
        uint32_t incl = len;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        const uint32_t span_bits = __shfl(incl, 63, 64);
        const uint32_t off = incl - len;
        const uint64_t rel0 = sync_base[g] - (word_base << 5);   // group start, bits from in[0]
        const uint64_t w0 = (rel0 >> 5) & ~3ull;                  // 16-B aligned staging origin
        const uint32_t lead = (uint32_t)(rel0 - (w0 << 5));        // bits before the group start
        const uint32_t nwords = (lead + span_bits + 31) / 32 + 2;  // + window look-ahead
        const uint64_t sym0 = c * S;
        const uint32_t cnt = valid ? (uint32_t)((n - sym0 < S) ? (n - sym0) : S) : 0u;
        const uint32_t pos = lead + off;                           // lane start, bits into staging
        uint8_t *row = ostage + lane * DEC_OUT_STRIDE;
        if (nwords + 1 <= DEC_STAGE_WORDS) {   // +1: the reader peeks one word ahead
            const uint4 *src = reinterpret_cast<const uint4 *>(in + w0);
            uint4 *dst = reinterpret_cast<uint4 *>(stage);
            const uint32_t nvec = (nwords + 4) / 4;
            // all loads in flight (named registers; indices clamped rather than loads
            // predicated, which made hipcc emit serialised flat loads), then byte-swapped
            // LDS writes
            static_assert((DEC_STAGE_WORDS / 4 + 63) / 64 <= 5, "stage larger than 5 KiB");
            const uint32_t i0 = lane, i1 = lane + 64, i2 = lane + 128, i3 = lane + 192, i4 = lane + 256,
                           last = nvec - 1;
            const uint4 v0 = src[min(i0, last)], v1 = src[min(i1, last)], v2 = src[min(i2, last)],
                        v3 = src[min(i3, last)], v4 = src[min(i4, last)];
#define DC_SWZ(v) make_uint4(bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w))
            if (i0 < nvec) dst[i0] = DC_SWZ(v0);
            if (i1 < nvec) dst[i1] = DC_SWZ(v1);
            if (i2 < nvec) dst[i2] = DC_SWZ(v2);
            if (i3 < nvec) dst[i3] = DC_SWZ(v3);
            if (i4 < nvec) dst[i4] = DC_SWZ(v4);
#undef DC_SWZ
            __builtin_amdgcn_wave_barrier();
            if (valid) {
                LdsWords rd{stage + (pos >> 5), 0u};
                if (stage_out) decode_chunk_lds(rd, pos & 31, cnt, row, L, T, nary, w, pow2, bad);
                else decode_chunk_hbm(rd, pos & 31, cnt, out + sym0, L, T, nary, w, pow2, bad);
            }
        } else if (valid) {
            HbmWords rd{in + w0 + (pos >> 5), 0u};
            if (stage_out) decode_chunk_lds(rd, pos & 31, cnt, row, L, T, nary, w, pow2, bad);
            else decode_chunk_hbm(rd, pos & 31, cnt, out + sym0, L, T, nary, w, pow2, bad);
        }
        if (stage_out) {
            // the group's 64 chunks are one contiguous output range: coalesced 16-B stores,
            // 1 KiB per wave-instruction (rows are 8-B aligned: two ds_read_b64 per piece)
            __builtin_amdgcn_wave_barrier();
            const uint64_t gbase = g * DC_SYNC_GROUP * (uint64_t)S;
            const uint64_t gbytes = (n - gbase < DC_SYNC_GROUP * (uint64_t)S) ? n - gbase : DC_SYNC_GROUP * (uint64_t)S;
            const uint32_t ppr_log = (uint32_t)__builtin_ctz(S) - 4;   // 16-B pieces per row, S power of two
            for (uint32_t j = lane; j < (uint32_t)(gbytes / 16); j += 64) {
                const uint32_t r = j >> ppr_log, q = j & ((1u << ppr_log) - 1);
                const uint64_t *src = reinterpret_cast<const uint64_t *>(ostage + r * DEC_OUT_STRIDE + q * 16);
                const uint64_t a = src[0], b = src[1];
                *reinterpret_cast<uint4 *>(out + gbase + (uint64_t)j * 16) =
                    make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
            }
            for (uint32_t k = (uint32_t)(gbytes & ~15ull) + lane; k < (uint32_t)gbytes; k += 64)
                out[gbase + k] = ostage[(k >> slog) * DEC_OUT_STRIDE + (k & (S - 1))];
        }
        __builtin_amdgcn_wave_barrier();   // staging areas reused by the next group
    }
    if (bad) atomicOr(err, 1);
}

// ------------------------------------------------------------------------------------
// (H8) decode, fast path for the default sync granularity S = 64 (k_huff_decode8).
// Same stream, same sync index, same output as k_huff_decode; built for ILP instead of
// per-step latency:
//  * staged words are bit-reversed within each byte (bfrev(bswap(w))), which turns the
//    MSB-first stream into an LSB-first one: stream bits [c, c+64) are two v_alignbit of
//    three consecutive words at c>>5, so a refill has no state but c;
//  * a lane decodes exactly 64 symbols per chunk, so every loop is fully unrolled with a
//    fixed trip count: no divergence, no loop control, and the output byte of symbol k
//    lands in register k/4 (v_perm); the lane's 64 output bytes stay in registers;
//  * batches of 4 symbols share one 64-bit window; a symbol is one v_lshrrev_b64, a
//    12-bit index and one 16-bit LUT read (len | sym << 8);
//  * several chains per lane (consecutive groups) are interleaved symbol by symbol (ILP);
//  * codes of 13..12+K bits (K <= 8): the first-level entry names a second-level table
//    indexed by the next K bits (rare, wave-uniform branch per symbol pair); anything
//    rarer (longer codes, a batch whose codes overflow the 64-bit window, invalid codes)
//    makes the wave redo its two chunks exactly (d8_chunk_hbm).
// Partial groups and groups whose span exceeds the stage also go through d8_chunk_hbm.
// ------------------------------------------------------------------------------------
#define D8_CHAINS 22           /* chains (groups being decoded) per CU: waves x chains/wave */
#define D8_LUT_BITS 15         /* first-level table of the fast decoder (64 KiB of LDS)      */
#define D8F_LUT_BITS 14        /* first level of the exact redo (32 KiB of LDS)             */
#define D8_STAGE_WORDS 1088    /* per chain: 4352 B = 4096 symbols at <= 8.4 bits/symbol   */
#define D8_L2_CAP 7168         /* second-level entries (u16)                               */
#define D8_K_MAX 8
#define D8_MAX_WAVES 16

struct Dec8Lds {
    __attribute__((aligned(16))) uint16_t lut[1 << D8_LUT_BITS];   // LSB-first 15-bit window -> len | sym << 8; len 0: a longer code
    uint32_t exhausted;               // scheduler: bit h = slice h is empty
    __attribute__((aligned(16))) uint32_t stage[D8_CHAINS][D8_STAGE_WORDS];
    uint32_t tail_pad[64];            // a corrupt stream's windows may run past the last stage
};

static __device__ __forceinline__ uint32_t brev8(uint32_t v) { return __builtin_bitreverse32(__builtin_bswap32(v)); }
// max of the two 16-bit halves separately (v_pk_max_u16)
static __device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const u16x2 r = __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b));
    return __builtin_bit_cast(uint32_t, r);
}


// exact slow decode of the code at the start of an LSB-first 64-bit window (lo, hi):
// returns nbits | sym << 8; an invalid code sets *bad and returns 0
static __device__ uint32_t d8_long(uint32_t lo, uint32_t hi, const dc_dtable *__restrict__ T, int nary, int w,
                                   bool pow2, int *bad)
{
    const uint64_t win = ((uint64_t)__builtin_bitreverse32(lo) << 32) | __builtin_bitreverse32(hi);   // MSB-first
    if (pow2) {
        const uint64_t top = win >> 32;
        uint32_t b = 1;
        while (b <= 32 && top >= T->lim[b]) ++b;
        if (b > 32) { *bad = 1; return 0u; }
        const uint32_t Ld = b / (uint32_t)w;
        const uint32_t v = (uint32_t)(top >> (32 - b));
        return b | ((T->syms[(T->start[Ld] + (v - T->first[Ld])) & (DC_MAX_SYMS - 1)] & 255u) << 8);
    }
    uint64_t x = win;
    uint32_t v = 0;
    for (int Ld = 1; Ld <= DC_MAX_DIGITS && Ld * w <= 32; ++Ld) {
        v = v * (uint32_t)nary + (uint32_t)(x >> (64 - w));
        x <<= w;
        const uint32_t cnt = T->count[Ld];
        if (cnt && v - T->first[Ld] < cnt) return (uint32_t)(Ld * w) | ((T->syms[T->start[Ld] + (v - T->first[Ld])] & 255u) << 8);
    }
    *bad = 1;
    return 0u;
}


// any chunk, any count, exact: words read from HBM (MSB-first bytes; reads clamped to the
// nwords of the buffer), bytes written one by one
static __device__ void d8_chunk_hbm(const uint32_t *__restrict__ in, uint64_t nwords, uint64_t pos, uint32_t cnt,
                                    uint8_t *__restrict__ o, const dc_dtable *__restrict__ T, int nary, int w,
                                    bool pow2, int &bad)
{
    for (uint32_t i = 0; i < cnt; ++i) {
        const uint64_t a = pos >> 5;
        if (a >= nwords) { bad = 1; return; }
        const uint32_t s = (uint32_t)pos & 31u;
        const uint32_t w0 = brev8(in[a]), w1 = brev8(in[min(a + 1, nwords - 1)]), w2 = brev8(in[min(a + 2, nwords - 1)]);
        const uint32_t e = d8_long(__builtin_amdgcn_alignbit(w1, w0, s), __builtin_amdgcn_alignbit(w2, w1, s), T, nary,
                                   w, pow2, &bad);
        if (e == 0) return;   // invalid code: stop this chunk (status reported)
        o[i] = (uint8_t)(e >> 8);
        pos += e & 255u;
    }
}

// Register window of a chain: 2 stage qwords q0:q1 in VGPRs and
// the window's bit position qb in them (0..63). A batch's 64-bit window is a funnel shift of
// q0:q1 (no stage read on the chain); the qword after q1 is read at the batch start, while
// the 4 lookups run, and when the batch's codes carry qb past 64 it moves in (q0 <- q1 <- it)
// by selects. One ds_read_b64 per batch where the r2 batch read 3 words at random banks
// (0.75 LDS reads per symbol, ~5.2 LDS cycles per symbol with their ~3.5-way conflicts:
// about 40% of the kernel's LDS cycles, profiles/r2k_pmc.txt). (An exec-masked read only
// where a lane needs it measured worse in code: the compiler waited for it inside the branch
// and the 16 unrolled branches cost 168 VGPRs with spills.)
template <int NC>
struct D8Win {
    uint64_t q0[NC], q1[NC];
    uint32_t qb[NC], qp[NC];   // bit position in q0:q1, index of the qword after q1
};

// chain start at stage bit P (a row of 64-bit words, 8-B aligned). 4 VALU + 1 LDS read per
// symbol: the window starts one bit early (the bit below the chunk's is a don't-care), so
// (win >> off) & (2^16 - 2) is the entry's byte address (no index scaling); the whole entry
// (len | sym << 8) is added to off, whose low 6 bits (all v_lshrrev_b64 reads) are then the
// bits consumed (the lengths of a batch sum to < 64, so they never carry into bit 8); an entry
// of no code is 0 (dlut15 escapes are zeroed), so min over the entries finds it. The window
// starts at P' - 64 with P' = P + 63: q0 = qword P'/64 - 1, which for
// P < 1 is the 8 bytes before the row (LDS in bounds: the previous row's tail, or the
// scheduler word and padding before the first row; a don't-care bit)
template <int NC>
static __device__ __forceinline__ void d8_win_init(D8Win<NC> &w, const uint64_t *const *st, const uint32_t *P)
{
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        const uint32_t p = P[j] + 63u, a = p >> 6;
        w.q0[j] = st[j][(int)a - 1];
        w.q1[j] = st[j][a];
        w.qb[j] = p & 63u;
        w.qp[j] = a + 1;
    }
}

template <int NC>
static __device__ __forceinline__ void d8_batch_q(const uint64_t *const *st, D8Win<NC> &w, uint32_t *o,
                                                  const uint16_t *__restrict__ lut, uint32_t *mn)
{
    uint64_t win[NC], nx[NC];
    uint32_t off[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        nx[j] = st[j][w.qp[j]];   // in flight during the lookups
        const uint32_t W0 = (uint32_t)w.q0[j], W1 = (uint32_t)(w.q0[j] >> 32);
        const uint32_t W2 = (uint32_t)w.q1[j], W3 = (uint32_t)(w.q1[j] >> 32);
        const bool k = w.qb[j] >= 32u;
        const uint32_t A = k ? W1 : W0, B = k ? W2 : W1, Cw = k ? W3 : W2;
        win[j] = ((uint64_t)__builtin_amdgcn_alignbit(Cw, B, w.qb[j]) << 32) | __builtin_amdgcn_alignbit(B, A, w.qb[j]);
        off[j] = 0;
    }
    const char *const lb = reinterpret_cast<const char *>(lut);
    constexpr uint32_t SEL[4] = {0x0c0c0c05u, 0x0c0c0500u, 0x0c050100u, 0x05020100u};
    uint32_t e[NC][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const uint32_t x = (uint32_t)(win[j] >> (off[j] & 63u));
            e[j][k] = *reinterpret_cast<const uint16_t *>(lb + (x & ((2u << D8_LUT_BITS) - 2u)));
            o[j] = __builtin_amdgcn_perm(e[j][k], k ? o[j] : 0u, SEL[k]);
            off[j] += e[j][k];
        }
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        mn[j] = min(mn[j], min(min(e[j][0], e[j][1]), min(e[j][2], e[j][3])));
        // a batch takes <= 60 bits (4 codes of <= 15), so qb < 124: one qword at most
        const uint32_t qb = w.qb[j] + (off[j] & 255u);
        const bool r = qb >= 64u;
        w.q0[j] = r ? w.q1[j] : w.q0[j];
        w.q1[j] = r ? nx[j] : w.q1[j];
        w.qp[j] += r ? 1u : 0u;
        w.qb[j] = qb & 63u;
    }
}

// The 16 batches of a 64-symbol chunk (4 pieces of 16 B per lane), unrolled by template
// recursion; the pieces stay in registers until the chunk is done.
template <int NC, int Q>
struct D8PiecesQ {
    static __device__ __forceinline__ void run(const uint64_t *const *st, D8Win<NC> &w, uint32_t (*o)[16],
                                               const uint16_t *__restrict__ lut, uint32_t *mn)
    {
        uint32_t b[NC];
        d8_batch_q<NC>(st, w, b, lut, mn);
#pragma unroll
        for (int j = 0; j < NC; ++j) o[j][Q] = b[j];
        D8PiecesQ<NC, Q + 1>::run(st, w, o, lut, mn);
    }
};
template <int NC>
struct D8PiecesQ<NC, 16> {
    static __device__ __forceinline__ void run(const uint64_t *const *, D8Win<NC> &, uint32_t (*)[16],
                                               const uint16_t *__restrict__, uint32_t *)
    {
    }
};

// A lane's 64 decoded bytes belong to its own chunk (lane = chunk): stored from registers,
// every wave store would touch 32 cache lines with 32 B each, and the L2 request rate then
// bounds the decoder (a contiguous-store ablation ran 0.72 -> 0.48 ms on 1 GiB C2). So the
// chain's 4 KiB of output go through its LDS stage, which the decode no longer needs: each
// lane writes its 4 pieces as a row (piece slots XOR-swizzled by lane so the 16-B writes of
// 8 lanes hit 8 distinct bank groups), then every store moves 1 KiB of contiguous output.
template <int NC>
static __device__ __forceinline__ void d8_out(uint32_t *const *stw, const uint32_t (*o)[16], uint4 *const *dst,
                                              int lane)
{
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        uint4 *row = reinterpret_cast<uint4 *>(stw[j]) + lane * 4;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            row[q ^ ((lane >> 1) & 3)] = make_uint4(o[j][4 * q], o[j][4 * q + 1], o[j][4 * q + 2], o[j][4 * q + 3]);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        const uint4 *rows = reinterpret_cast<const uint4 *>(stw[j]);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const uint32_t ch = 16 * s + (lane >> 2), p = lane & 3;
            const uint4 v = rows[ch * 4 + (p ^ ((ch >> 1) & 3))];
            // streaming (nt) stores: the decoded output is not read again here, and written
            // back at once it leaves no dirty lines for the next kernels' reads to evict
            // (1 GiB C2 step, same-box A/B: the next histogram 0.244 -> 0.208 ms, the decode
            // itself 0.432 -> 0.420, the redo 0.046 -> 0.038)
            __builtin_nontemporal_store(v.x, &dst[j][s * 64 + lane].x);
            __builtin_nontemporal_store(v.y, &dst[j][s * 64 + lane].y);
            __builtin_nontemporal_store(v.z, &dst[j][s * 64 + lane].z);
            __builtin_nontemporal_store(v.w, &dst[j][s * 64 + lane].w);
        }
    }
}


typedef __attribute__((address_space(4))) const uint64_t c_u64;   // scalar (s_load) reads

template <int NC>
struct D8Meta { uint32_t len[NC]; uint64_t base[NC]; };   // sync index of one tuple: len per lane, base uniform
template <int NC>
struct D8Geo {            // where a tuple's spans and chunks lie; all uniform except off
    uint32_t g0;          // first group
    uint32_t wo[NC];      // first staged word (16-B aligned), relative to word_base
    uint32_t lead[NC];    // stage bit of the group's first chunk
    uint32_t last[NC];    // last uint4 of the stage
    uint32_t off[NC];     // this lane's chunk: bit offset inside the group span
    bool fast;
};

template <int NC>
static __device__ __forceinline__ void d8_load_meta(D8Meta<NC> &m, uint32_t tp, uint32_t ngroups, uint32_t nchunks,
                                                    int lane, const uint16_t *__restrict__ sync_len,
                                                    const uint64_t *__restrict__ sync_base)
{
    // unconditional loads of clamped indices: a conditional load would make the compiler
    // wait for it (and for every older load: the prefetched spans) at the join; the
    // validity mask is applied where the values are used, an iteration later. The group
    // bases are wave-uniform: scalar loads (lgkmcnt, SGPRs), no vector registers.
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        const uint32_t g = tp * NC + j, ch = g * DC_SYNC_GROUP + lane;
        m.len[j] = sync_len[min(ch, nchunks - 1)];
        m.base[j] = ((c_u64 *)sync_base)[min(g, ngroups - 1)];
    }
}

template <int NC>
static __device__ __forceinline__ void d8_geometry(D8Geo<NC> &g, const D8Meta<NC> &m, uint32_t tp, uint32_t ntuples,
                                                   uint64_t n, uint32_t nchunks, uint64_t nwords, uint64_t word_base,
                                                   int lane)
{
    constexpr uint64_t GSYM = DC_SYNC_GROUP * 64;
    g.g0 = tp * NC;
    uint32_t in[NC], len[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {   // branch-free mask (a branch here makes the compiler drain vmcnt)
        const uint32_t ok = (uint32_t)(tp < ntuples) & (uint32_t)((g.g0 + j) * DC_SYNC_GROUP + lane < nchunks);
        len[j] = m.len[j] & (0u - ok);
        in[j] = len[j];
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) in[j] = wave_scan_incl(in[j]);
    bool fast = tp < ntuples && (uint64_t)(g.g0 + NC) * GSYM <= n;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        const uint32_t span = __builtin_amdgcn_readlane(in[j], 63);
        g.off[j] = in[j] - len[j];
        const uint64_t rel = m.base[j] - (word_base << 5);
        g.wo[j] = (uint32_t)(rel >> 5) & ~3u;
        g.lead[j] = (uint32_t)rel & 127u;
        const uint32_t nw = (g.lead[j] + span) / 32 + 3;
        g.last[j] = (nw + 3) / 4 - 1;
        fast = fast && nw + 4 <= D8_STAGE_WORDS && (uint64_t)g.wo[j] + nw + 4 <= nwords;
    }
    g.fast = fast;
}

// the tuple's span loads: 16 B per lane, clamped to each span; word 0 when not staged
template <int NC>
static __device__ __forceinline__ void d8_issue(uint4 (&v)[NC][5], const D8Geo<NC> &g,
                                                const uint32_t *__restrict__ in, int lane)
{
#pragma unroll
    for (int k = 0; k < 5; ++k) {
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const uint4 *src = reinterpret_cast<const uint4 *>(in + (g.fast ? g.wo[j] : 0u));
            v[j][k] = LD_DEC(src + (g.fast ? min((uint32_t)(lane + 64 * k), g.last[j]) : 0u));
        }
    }
}

// Tuple scheduler of the persistent decoder. Waves of one SIMD get unequal issue slots
// (priority, then age) and XCDs run at slightly different speeds, so a static split ends
// when the slowest wave does (measured 1.5x max/min inside a workgroup). The first
// D8_STATIC_PCT % of the tuples are dealt statically (wave i: i, i + P, i + 2P, ...); the
// rest are cut into 8 slices, each with its own dequeue head (a u32 counter on a 4 KiB
// line of its own: one word saturates at ~88 dequeues/us, MI355X_MICROARCH.md 'dequeue').
// A wave dequeues from the slice of its block's group label (blockIdx % 8), then steals
// from the other slices; a workgroup remembers exhausted slices in LDS. The last wave out
// resets the heads for the next launch on the stream.
#define D8_STATIC_PCT 60
#define D8_QSTRIDE 1024   /* u32 between heads */
#define D8_QWORDS (11 * D8_QSTRIDE)

struct D8Sched {
    uint32_t Ts, Dh, ntuples;   // static tuples, slice size, all tuples
    uint32_t wid, P;            // wave id, waves in the grid
    uint32_t k, Ks;             // static tuples taken / per wave
    int head, tried;            // slice being drained, slices given up
    bool dyn;                   // pending value is a dequeue result
    uint32_t pend;              // lane 0: dequeued index
    uint32_t spend;             // static index
};

static __device__ __forceinline__ void d8_fetch(D8Sched &s, uint32_t *__restrict__ queue, int lane)
{
    if (s.k < s.Ks) {
        s.spend = s.wid + s.k * s.P;
        ++s.k;
        s.dyn = false;
    } else {
        s.dyn = true;
        if (lane == 0 && s.tried < 8) s.pend = atomicAdd(queue + s.head * D8_QSTRIDE, 1u);
    }
}

// a dequeued index past its slice: mark the slice empty, then probe the others in turn
static __device__ uint32_t d8_resolve_retry(D8Sched &s, uint32_t *__restrict__ queue, uint32_t *exhausted, int lane)
{
    while (s.tried < 8) {
        if (lane == 0) atomicOr(exhausted, 1u << s.head);
        ++s.tried;
        s.head = (s.head + 1) & 7;
        // skip slices this workgroup already found empty
        const uint32_t ex = __builtin_amdgcn_readfirstlane(__atomic_load_n(exhausted, __ATOMIC_RELAXED));
        while (s.tried < 8 && ((ex >> s.head) & 1u)) { ++s.tried; s.head = (s.head + 1) & 7; }
        if (s.tried >= 8) break;
        if (lane == 0) s.pend = atomicAdd(queue + s.head * D8_QSTRIDE, 1u);
        const uint32_t i = (uint32_t)__builtin_amdgcn_readlane((int)s.pend, 0);
        const uint32_t lo = s.Ts + (uint32_t)s.head * s.Dh;
        const uint32_t hi = min(lo + s.Dh, s.ntuples);
        if (i < hi - min(lo, hi)) return lo + i;
    }
    return s.ntuples;
}

// The common case is loop-free, so the compiler's wait for the dequeue issued an iteration
// earlier counts only the ops issued since (spans, output stores): vmcnt(N), not vmcnt(0)
// (a loop here would make it drain every outstanding store first).
static __device__ __forceinline__ uint32_t d8_resolve(D8Sched &s, uint32_t *__restrict__ queue, uint32_t *exhausted,
                                                      int lane)
{
    if (!s.dyn) return s.spend;
    if (s.tried < 8) {
        const uint32_t i = (uint32_t)__builtin_amdgcn_readlane((int)s.pend, 0);
        const uint32_t lo = s.Ts + (uint32_t)s.head * s.Dh;
        const uint32_t hi = min(lo + s.Dh, s.ntuples);
        if (i < hi - min(lo, hi)) return lo + i;
    }
    return d8_resolve_retry(s, queue, exhausted, lane);
}

// byte-wise bit reversal of a tuple's spans (registers) into its LDS stage rows
template <int NC>
static __device__ __forceinline__ void d8_stage(const D8Geo<NC> &cur, const uint4 (&v)[NC][5], uint32_t *const *stw,
                                                int lane)
{
    if (!cur.fast) return;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t i = lane + 64 * k;
#pragma unroll
        for (int j = 0; j < NC; ++j)
            if (i <= cur.last[j])
                reinterpret_cast<uint4 *>(stw[j])[i] =
                    make_uint4(brev8(v[j][k].x), brev8(v[j][k].y), brev8(v[j][k].z), brev8(v[j][k].w));
    }
}

// A fast decoder that finds its tables stale (dec_ready 0: the table was rewritten since
// they were built) reports a stream error and decodes nothing. The launches after it must
// then find nothing to redo: workgroup 0 zeroes the redo counter, every workgroup zeroes its
// grid-stride share of the groups' redo masks, and every wave still counts itself out of the
// scheduler (the last one out resets the dequeue heads), so the next decode on this context
// starts clean even when only some workgroups took this exit.
static __device__ void d8_stale_exit(int *__restrict__ err, uint32_t *__restrict__ queue,
                                     uint64_t *__restrict__ fix_mask, uint64_t n, int nw)
{
    const int t = threadIdx.x;
    if (t == 0) atomicOr(err, 1);
    const uint64_t ngroups = ((n + 63) / 64 + DC_SYNC_GROUP - 1) / DC_SYNC_GROUP;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + t; g < ngroups; g += (uint64_t)gridDim.x * blockDim.x)
        fix_mask[g] = 0ull;
    if ((t & 63) == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (atomicAdd(queue + 8 * D8_QSTRIDE, 1u) == gridDim.x * (uint32_t)nw - 1)
            for (int h = 0; h <= 8; ++h) atomicExch(queue + h * D8_QSTRIDE, 0u);
    }
}

// NW waves per workgroup (one workgroup per CU), NC chains per wave: wave w of workgroup b
// decodes the NC consecutive groups of "tuple" b*NW + w (+ grid stride), lane = chunk.
// EXP (the C5 decode, dc_small_huff_decode): also the number of symbols >= 0x80 of every group
// into gexp[group] (each is a front-end pair: two output bytes), so the front-end inverse needs
// no counting pass of its own; the redo adds those of the chunks it rewrites.
template <int NW, int NC, bool EXP = false>
__global__ __launch_bounds__(NW * 64) void k_huff_decode8(const uint32_t *__restrict__ in, uint64_t bit_base, const uint64_t *__restrict__ d_base,
                                                          const uint64_t *__restrict__ sync_base,
                                                          const uint16_t *__restrict__ sync_len, uint64_t n,
                                                          uint64_t nwords, const dc_dtable *__restrict__ T,
                                                          uint8_t *__restrict__ out, int *__restrict__ err,
                                                          uint32_t *__restrict__ queue, uint32_t static_pct,
                                                          uint64_t *__restrict__ fix_mask, uint64_t *__restrict__ fix_pos,
                                                          uint8_t *__restrict__ scratch, uint32_t *__restrict__ gexp = nullptr)
{
    static_assert(NW * NC <= D8_CHAINS && NW <= D8_MAX_WAVES, "stage slots");
    constexpr uint32_t S = 64;
    constexpr int NT = NW * 64;
    __shared__ Dec8Lds L;
    if (!__hip_atomic_load(&T->dec_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {   // tables rebuilt since
        // reported as a stream error; the redo launches that follow must find nothing to do
        d8_stale_exit(err, queue, fix_mask, n, NW);
        return;
    }
    if (d_base) bit_base += *d_base;   // device-resident shard offset (dist: no host read)
    if (!EXP && T->fixed8 && (bit_base & 127) == 0 && ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
        (n + 3) / 4 <= nwords) {
        // every code 8 bits: output symbol i = the symbol of stream byte bit_base / 8 + i (the
        // words' first byte; bit_base % 128 == 0). No chunk is redone: the fix masks are zeroed.
        uint16_t *const inv = reinterpret_cast<uint16_t *>(L.lut);   // byte -> symbol, 0x100 = no code
        const int tt = threadIdx.x;
        for (int i = tt; i < 256; i += NW * 64) inv[i] = 0x100;
        __syncthreads();
        for (int sy = tt; sy < 256; sy += NW * 64)
            if (T->nbits[sy] == 8u) inv[T->code[sy] & 255u] = (uint16_t)sy;
        __syncthreads();
        const uint8_t *const ib = reinterpret_cast<const uint8_t *>(in);
        const uint64_t nthr = (uint64_t)gridDim.x * NW * 64, me = (uint64_t)blockIdx.x * NW * 64 + tt;
        uint32_t bad = 0;
        // affine (dc_dtable.fixed8_affine): symbol = code + lo for codes 0 .. count - 1; a code past
        // them (the dummy leaves' codes) is a stream error: the largest code byte, kept per 16-bit
        // lane by v_pk_max_u16 on the even and the odd bytes, is checked once at the end
        const bool aff = T->fixed8_affine != 0;
        const uint32_t lo4 = (uint32_t)(T->fixed8_lo & 255) * 0x01010101u;
        uint32_t cmax = 0;
        // 4 granules a thread per round, their loads issued together: one workgroup of NW waves
        // per CU (the decoder's launch) keeps too few loads in flight with one
        const uint64_t ng = n / 16;
        auto put = [&](uint64_t g, const uint32_t (&w4)[4]) {   // streaming stores, as d8_out
            uint4 *const o4 = reinterpret_cast<uint4 *>(out + 16 * g);
            __builtin_nontemporal_store(w4[0], &o4->x);
            __builtin_nontemporal_store(w4[1], &o4->y);
            __builtin_nontemporal_store(w4[2], &o4->z);
            __builtin_nontemporal_store(w4[3], &o4->w);
        };
        for (uint64_t g0 = me; g0 < ng; g0 += 4 * nthr) {
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint64_t g = g0 + (uint64_t)u * nthr;
                v[u] = g < ng ? LD_DEC(reinterpret_cast<const uint4 *>(ib + 16 * g)) : make_uint4(0u, 0u, 0u, 0u);
            }
            if (aff) {   // no byte carries: a valid code + lo is a byte
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        cmax = pk_max_u16(cmax, w4[q] & 0x00FF00FFu);
                        cmax = pk_max_u16(cmax, (w4[q] >> 8) & 0x00FF00FFu);
                        w4[q] += lo4;
                    }
                    const uint64_t g = g0 + (uint64_t)u * nthr;
                    if (g < ng) put(g, w4);
                }
            } else {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint32_t x = w4[q];
                        const uint32_t a = inv[x & 255u], b2 = inv[(x >> 8) & 255u], c2 = inv[(x >> 16) & 255u], d2 = inv[x >> 24];
                        bad |= (a | b2 | c2 | d2) & 0x100u;
                        w4[q] = (a & 255u) | ((b2 & 255u) << 8) | ((c2 & 255u) << 16) | ((d2 & 255u) << 24);
                    }
                    const uint64_t g = g0 + (uint64_t)u * nthr;
                    if (g < ng) put(g, w4);
                }
            }
        }
        for (uint64_t i = (n & ~15ull) + me; i < n; i += nthr) {
            const uint32_t a = inv[ib[i]];
            bad |= a & 0x100u;
            out[i] = (uint8_t)a;
        }
        const uint32_t cm = max(cmax & 0xFFFFu, cmax >> 16);
        if (aff && cm >= (uint32_t)T->fixed8_count) bad = 1;
        if (bad) atomicOr(err, 1);
        const uint32_t ngr = (uint32_t)(((n + S - 1) / S + DC_SYNC_GROUP - 1) / DC_SYNC_GROUP);
        for (uint64_t g = me; g < ngr; g += nthr) fix_mask[g] = 0ull;
        return;
    }
    const int t = threadIdx.x, lane = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    // ---- table: the LSB-first 12-bit table (dc_dtable.dlut); codes longer than 12 bits
    // read length 0
    // D8_LUT_BITS first level from the 12-bit one and its second level: 2.9% of C2 chunks hold a
    // code of > 14 bits (to the exact redo), 6.6% one of > 12
    // the 15-bit first level (dc_dtable.dlut15, built by dec_tables_build): 1.2% of C2 chunks
    // hold a code of > 15 bits (to the exact redo; 2.5% with the 14-bit table of r1)
    static_assert(D8_LUT_BITS == DC_LUT15_BITS, "table width");
    for (int i = t; i < (1 << D8_LUT_BITS) / 8; i += NT)
        reinterpret_cast<uint4 *>(L.lut)[i] = reinterpret_cast<const uint4 *>(T->dlut15)[i];
    if (t == 0) L.exhausted = 0;
    __syncthreads();

    // the launcher guarantees n < 2^37 (chunk and tuple indices fit 32 bits)
    const uint32_t nchunks = (uint32_t)((n + S - 1) / S);
    const uint32_t ngroups = (nchunks + DC_SYNC_GROUP - 1) / DC_SYNC_GROUP;
    const uint32_t ntuples = (ngroups + NC - 1) / NC;
    const uint64_t word_base = bit_base >> 5;
    uint32_t *stw[NC];
    const uint64_t *st64[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        stw[j] = L.stage[wv * NC + j];
        st64[j] = reinterpret_cast<const uint64_t *>(stw[j]);
    }
    const uint32_t stride = gridDim.x * NW;
    // Software pipeline (per wave, one tuple of NC groups per iteration): while tuple i
    // decodes, the spans of tuple i+1 are in flight into registers and the sync index of
    // tuple i+2 too, so no iteration waits for a global round trip.
    // The span loads are issued for every tuple (clamped to word 0 when it is not staged),
    // so the prefetch registers never need merging.
    static_assert((D8_STAGE_WORDS / 4 + 63) / 64 <= 5, "stage larger than 5 KiB");
    D8Geo<NC> g, cur;
    D8Meta<NC> m1, m2;   // m2: the first tuple's index only
    uint4 v[NC][5];
    D8Sched sc;
    sc.ntuples = ntuples;
    sc.P = stride;
    sc.wid = blockIdx.x * NW + wv;
    sc.Ks = (uint32_t)((uint64_t)ntuples * static_pct / 100 / stride);
    sc.Ts = sc.Ks * stride;
    sc.Dh = (ntuples - sc.Ts + 7) / 8;
    sc.k = 0;
    sc.head = blockIdx.x & 7;
    sc.tried = 0;
    sc.pend = 0;
    d8_fetch(sc, queue, lane);
    uint32_t tp = d8_resolve(sc, queue, &L.exhausted, lane);
    d8_fetch(sc, queue, lane);
    uint32_t t1 = d8_resolve(sc, queue, &L.exhausted, lane);
    d8_fetch(sc, queue, lane);
    // Rotated software pipeline (per wave): the loop body decodes the staged tuple, then
    // stages the next one from registers and issues the loads of the one after. The span
    // loads are thereby always older than the decode's 32 output stores (vector memory ops
    // retire in issue order), so staging waits for vmcnt(32), not for the stores to drain.
    // That needs the 32 stores on every path: a tuple the fast decoder cannot take (partial
    // group, over-long span) still runs it, on whatever the stage holds, with its stores sent
    // to the trash rows wherever a chunk is not whole inside the output; the exact redo
    // rewrites the real bytes afterwards (same wave, program order).
    // per-wave scratch (garbage sinks): stores that land on lines every wave shares would
    // serialise in L2, so each wave has its own: 2 chains x 4 KiB of trash rows, 65 u64 dummies
    uint8_t *const wscr = scratch + (size_t)(blockIdx.x * NW + wv) * D8_WSCR;
    uint4 *const trash = reinterpret_cast<uint4 *>(wscr);
    uint32_t *const dummy = reinterpret_cast<uint32_t *>(wscr + 2 * 4096);
    d8_load_meta<NC>(m2, tp, ngroups, nchunks, lane, sync_len, sync_base);
    d8_geometry<NC>(g, m2, tp, ntuples, n, nchunks, nwords, word_base, lane);
    d8_issue<NC>(v, g, in, lane);
    d8_load_meta<NC>(m1, t1, ngroups, nchunks, lane, sync_len, sync_base);
    cur = g;
    d8_stage<NC>(cur, v, stw, lane);
    d8_geometry<NC>(g, m1, t1, ntuples, n, nchunks, nwords, word_base, lane);
    uint32_t t2 = d8_resolve(sc, queue, &L.exhausted, lane);
    d8_load_meta<NC>(m1, t2, ngroups, nchunks, lane, sync_len, sync_base);
    d8_fetch(sc, queue, lane);
    d8_issue<NC>(v, g, in, lane);
    while (tp < ntuples) {
        __builtin_amdgcn_wave_barrier();
        uint32_t c[NC];
        uint4 *dst[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            // the group's 4 KiB of output (d8_out); a tuple that is not fast (its chunks are
            // all rewritten by the redo) stores into the chain's trash rows instead
            c[j] = cur.fast ? cur.lead[j] + cur.off[j] : 0u;   // the chunk's stage bit
            dst[j] = cur.fast ? reinterpret_cast<uint4 *>(out + (uint64_t)(cur.g0 + j) * DC_SYNC_GROUP * S)
                              : trash + j * 256;
        }
        // mn[j] == 0 after the decode <=> chunk redone: starts at 0 for a tuple that is not
        // fast (the fixup skips chunks past the end), reaches 0 on a code of > 12 bits
        uint32_t o[NC][16], mn[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) mn[j] = cur.fast ? 255u : 0u;
        {
            D8Win<NC> wq;
            d8_win_init<NC>(wq, st64, c);
            D8PiecesQ<NC, 0>::run(st64, wq, o, L.lut, mn);
        }
        d8_out<NC>(stw, o, dst, lane);
        // chunks with a code of > 12 bits (and every chunk of a tuple that was not fast:
        // partial group, over-long span) are decoded again exactly by k_huff_decode8_fix:
        // a bit per chunk, and for those chunks their bit offset inside the group
        // (no branch: any exec-masked store in this loop body costs ~80 VGPRs of allocation,
        // so lanes without something to record write a per-lane dummy slot instead)
        // (cur.fast is not read after the decode either: that made the compiler keep two
        // versions of the whole decode live, 168 VGPRs + spills instead of 91)
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const uint32_t g = cur.g0 + j;
            const bool redo = mn[j] == 0;
            const uint64_t m = __ballot(redo);
            uint64_t *pp = redo ? fix_pos + (uint64_t)g * DC_SYNC_GROUP + lane : reinterpret_cast<uint64_t *>(dummy) + lane;
            *pp = (uint64_t)cur.wo[j] * 32 + cur.lead[j] + cur.off[j];   // chunk start, bits from word_base
            uint64_t *mp = g < ngroups ? fix_mask + g : reinterpret_cast<uint64_t *>(dummy) + 64;
            *mp = m;
            // the first flagged chunk's start also beside the masks (fix_mask + ngroups: the redo
            // reads it with them, coalesced, instead of gathering its fix_pos line)
            const uint32_t f = (uint32_t)__builtin_ctzll(m | (1ull << 63));
            uint64_t *fp = g < ngroups ? fix_mask + ngroups + g : reinterpret_cast<uint64_t *>(dummy) + 65;
            *fp = (uint64_t)cur.wo[j] * 32 + cur.lead[j] + (uint32_t)__builtin_amdgcn_readlane((int)cur.off[j], (int)f);
            if (EXP) {   // symbols >= 0x80 of the chunks not redone (the redo adds the others)
                uint32_t e = 0;
#pragma unroll
                for (int q = 0; q < 16; ++q) e += (uint32_t)__popc(o[j][q] & 0x80808080u);
                e = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_incl(redo ? 0u : e), 63);
                uint32_t *ep = (lane == 0 && g < ngroups) ? gexp + g : dummy + 132 + lane;
                *ep = e;
            }
        }
        // next tuple: stage it (its spans are in v), then start the loads of the one after
        tp = t1;
        t1 = t2;
        cur = g;
        __builtin_amdgcn_wave_barrier();   // the stage is rewritten
        d8_stage<NC>(cur, v, stw, lane);
        d8_geometry<NC>(g, m1, t1, ntuples, n, nchunks, nwords, word_base, lane);
        t2 = d8_resolve(sc, queue, &L.exhausted, lane);
        d8_load_meta<NC>(m1, t2, ngroups, nchunks, lane, sync_len, sync_base);
        d8_fetch(sc, queue, lane);
        d8_issue<NC>(v, g, in, lane);   // after the index loads: waiting for these covers both
    }
    if (lane == 0) {
        // a dequeue issued for a tuple past the end may still be in flight: it must land
        // before this wave counts itself out, or it would bump a head after the reset
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (atomicAdd(queue + 8 * D8_QSTRIDE, 1u) == gridDim.x * NW - 1)
            for (int h = 0; h <= 8; ++h) atomicExch(queue + h * D8_QSTRIDE, 0u);
    }
}


// The exact redo's LDS: the 14-bit table, its second level and the canonical tables of longer
// codes (d8_long's rule), and a span row per lane.
#ifndef D8F_WAVES
#define D8F_WAVES 16   /* 16 x 24-word rows: 0.113 -> 0.091 ms on 1 GiB C2 vs 12 x 32 */
#endif
#ifndef D8F_ROW
#define D8F_ROW 20   /* words of a lane's staged span (longer chunks re-stage it further on; r2-r3: 24) */
#endif
static_assert(offsetof(dc_dtable, dlut14) % 16 == 0 && offsetof(dc_dtable, dlut15) % 16 == 0 && offsetof(dc_dtable, dlut2) % 8 == 0,
              "table copies");
struct FixLds {
    __attribute__((aligned(16))) uint16_t lut[1 << D8F_LUT_BITS];   // the fast decoder's 14-bit first level
    uint16_t lut2[DC_LUT2_CAP];
    uint64_t lim[33];
    uint32_t first[DC_MAX_DIGITS + 1], count[DC_MAX_DIGITS + 1], start[DC_MAX_DIGITS + 1];
    uint16_t syms[DC_MAX_SYMS];
    uint32_t rows[D8F_WAVES][64 * (D8F_ROW + 1)];   // a lane's chunk span (odd stride: conflict-free)
};

// d8_long on the LDS copies: the code at the start of an LSB-first 64-bit window; 0 for an
// invalid code (out of line: rare, and inlined 4 times it cost 70 VGPRs)
static __device__ __noinline__ uint32_t d8_long_lds(uint32_t lo, uint32_t hi, const FixLds &F, int nary, int w, bool pow2)
{
    const uint64_t win = ((uint64_t)__builtin_bitreverse32(lo) << 32) | __builtin_bitreverse32(hi);   // MSB-first
    if (pow2) {
        const uint64_t top = win >> 32;
        uint32_t b = 1;
        while (b <= 32 && top >= F.lim[b]) ++b;
        if (b > 32) return 0u;
        const uint32_t Ld = b / (uint32_t)w;
        const uint32_t v = (uint32_t)(top >> (32 - b));
        return b | ((F.syms[(F.start[Ld] + (v - F.first[Ld])) & (DC_MAX_SYMS - 1)] & 255u) << 8);
    }
    uint64_t x = win;
    uint32_t v = 0;
    for (int Ld = 1; Ld <= DC_MAX_DIGITS && Ld * w <= 32; ++Ld) {
        v = v * (uint32_t)nary + (uint32_t)(x >> (64 - w));
        x <<= w;
        const uint32_t cnt = F.count[Ld];
        if (cnt && v - F.first[Ld] < cnt)
            return (uint32_t)(Ld * w) | ((F.syms[(F.start[Ld] + (v - F.first[Ld])) & (DC_MAX_SYMS - 1)] & 255u) << 8);
    }
    return 0u;
}

// Exact decode of the chunks k_huff_decode8 flagged (fix_mask: a bit per chunk, fix_pos: the
// chunk's first bit, from word_base), in one launch. Workgroup b takes an equal share of the
// groups' masks, a window of 1024 at a time (one per thread): popcounts, a workgroup scan, and
// the window's flagged chunks listed in LDS; its waves take the list in rounds of 64 (one
// chunk per lane): wave w rounds w, w + 16, ... While round A decodes from its LDS rows, the
// spans of round B are in flight into registers and the start position of round C too. Per
// symbol a two-level lookup (the fast decoder's 14-bit table, then the second level on the
// next K bits only when a lane needs it) and a canonical search only for codes past the
// second level. Output leaves as one u32 per 4 symbols straight to HBM (26 MB on 1 GiB C2).
// (r2 listed the chunks in a launch of its own, k_huff_fix_list: 0.008 ms + a launch gap on
// 1 GiB C2; a flagged chunk falls in any group with the same odds, so equal shares of the
// groups are equal shares of the work, ~12 rounds per workgroup of 16 waves on C2.)
#define D8F_LIST 1024   /* listed chunks per pass (LDS) */
__global__ __launch_bounds__(D8F_WAVES * 64) void k_huff_decode8_fix(const uint32_t *__restrict__ in, uint64_t n,
                                                                    uint64_t nwords, const dc_dtable *__restrict__ T,
                                                                    uint8_t *__restrict__ out, int *__restrict__ err,
                                                                    const uint64_t *__restrict__ fix_mask,
                                                                    const uint64_t *__restrict__ fix_pos,
                                                                    int *__restrict__ err_next, uint32_t *__restrict__ gexp = nullptr)
{
    constexpr uint32_t S = 64;
    constexpr int NT = D8F_WAVES * 64;
    __shared__ FixLds F;
    __shared__ uint32_t s_list[D8F_LIST];
    __shared__ uint64_t s_pos[D8F_LIST];   // a listed chunk's start when it is its group's first, else ~0
    __shared__ uint32_t s_wsum[D8F_WAVES];
    const int t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);
    if (blockIdx.x == 0 && t < 4) err_next[t] = 0;   // the next decode's error slot
    const uint32_t nchunks = (uint32_t)((n + S - 1) / S);
    const uint32_t ngroups = (nchunks + DC_SYNC_GROUP - 1) / DC_SYNC_GROUP;
    const uint32_t g0 = (uint32_t)((uint64_t)ngroups * blockIdx.x / gridDim.x);
    const uint32_t g1 = (uint32_t)((uint64_t)ngroups * (blockIdx.x + 1) / gridDim.x);
    const uint32_t K2 = (uint32_t)T->dlut2_k, kmask = (1u << K2) - 1;
    auto window_mask = [&](uint32_t g) -> uint64_t {   // chunks past the end are never redone
        uint64_t m = g < g1 ? fix_mask[g] : 0ull;
        const uint64_t c0 = (uint64_t)g * DC_SYNC_GROUP;
        if (c0 + DC_SYNC_GROUP > nchunks) m = c0 >= nchunks ? 0ull : m & ((1ull << (nchunks - c0)) - 1);
        return m;
    };
    const uint64_t *const fix_first = fix_mask + ngroups;   // (k_huff_decode8: the first flagged chunk's start)
    auto window_first = [&](uint32_t g) -> uint64_t { return fix_first[g < g1 ? g : g0]; };
    uint64_t mk = window_mask(g0 + t);   // the first window's masks, in flight during the table copy
    uint64_t fk = window_first(g0 + t);
    {   // the tables into LDS: all loads first, then the stores
        static_assert((1 << D8F_LUT_BITS) / 8 <= 2 * NT && DC_LUT2_CAP / 4 <= 2 * NT && DC_MAX_SYMS <= NT &&
                      DC_MAX_DIGITS + 1 <= NT, "one copy pass");
        const uint4 *l1 = reinterpret_cast<const uint4 *>(T->dlut14);
        const uint2 *l2 = reinterpret_cast<const uint2 *>(T->dlut2);   // dlut2 is 8-B aligned
        constexpr int N1 = (1 << D8F_LUT_BITS) / 8, N2 = DC_LUT2_CAP / 4;
        const uint4 a0 = l1[t], a1 = t + NT < N1 ? l1[t + NT] : make_uint4(0u, 0u, 0u, 0u);
        const uint2 b0 = t < N2 ? l2[t] : make_uint2(0u, 0u), b1 = t + NT < N2 ? l2[t + NT] : make_uint2(0u, 0u);
        const uint16_t sy = t < DC_MAX_SYMS ? T->syms[t] : (uint16_t)0;
        const bool cn = t <= DC_MAX_DIGITS;
        const uint32_t fi = cn ? T->first[t] : 0u, co = cn ? T->count[t] : 0u, sa = cn ? T->start[t] : 0u;
        const uint64_t li = t < 33 ? T->lim[t] : 0ull;
        reinterpret_cast<uint4 *>(F.lut)[t] = a0;
        if (t + NT < N1) reinterpret_cast<uint4 *>(F.lut)[t + NT] = a1;
        if (t < N2) reinterpret_cast<uint2 *>(F.lut2)[t] = b0;
        if (t + NT < N2) reinterpret_cast<uint2 *>(F.lut2)[t + NT] = b1;
        if (t < DC_MAX_SYMS) F.syms[t] = sy;
        if (cn) { F.first[t] = fi; F.count[t] = co; F.start[t] = sa; }
        if (t < 33) F.lim[t] = li;
    }
    const int nary = T->n_ary, w = T->w;
    const bool pow2 = (nary & (nary - 1)) == 0;
    uint32_t *row = F.rows[wv] + lane * (D8F_ROW + 1);
    int bad = 0;
    // a span's 16-B aligned first word (clamped so that a whole row can be read)
    auto row_base = [&](uint64_t pos) -> uint64_t {
        const uint64_t lim = nwords > D8F_ROW ? (nwords - D8F_ROW) & ~3ull : 0ull;
        return min((pos >> 5) & ~3ull, lim);
    };
    auto load_row = [&](uint4 (&v)[D8F_ROW / 4], uint64_t a0) {
        const uint64_t nq = (nwords - a0) / 4;
#pragma unroll
        for (int k = 0; k < D8F_ROW / 4; ++k)
            v[k] = (uint64_t)k < nq ? reinterpret_cast<const uint4 *>(in + a0)[k] : make_uint4(0u, 0u, 0u, 0u);
    };
    auto put_row = [&](const uint4 (&v)[D8F_ROW / 4]) {
#pragma unroll
        for (int k = 0; k < D8F_ROW / 4; ++k) {
            row[4 * k] = brev8(v[k].x);
            row[4 * k + 1] = brev8(v[k].y);
            row[4 * k + 2] = brev8(v[k].z);
            row[4 * k + 3] = brev8(v[k].w);
        }
    };
    for (uint32_t wb = g0; wb < g1; wb += NT) {
        // this window's flagged chunks: the thread of group g lists its chunks after those of
        // the groups before it
        const uint32_t c = (uint32_t)__popcll(mk);
        const uint32_t incl = wave_scan_incl(c);
        if (lane == 63) s_wsum[wv] = incl;
        __syncthreads();   // (also: the table copy, the previous window's rounds)
        uint32_t before = 0, total = 0;
#pragma unroll
        for (int q = 0; q < D8F_WAVES; ++q) {
            const uint32_t x = s_wsum[q];
            before += q < wv ? x : 0u;
            total += x;
        }
        const uint64_t m_me = mk, f_me = fk;
        const uint32_t c0 = (wb + (uint32_t)t) * DC_SYNC_GROUP;
        if (wb + NT < g1) {   // the next window's masks, in flight
            mk = window_mask(wb + NT + t);
            fk = window_first(wb + NT + t);
        }
        for (uint32_t part = 0; part < total; part += D8F_LIST) {   // (one part unless > 2048 chunks)
            {
                uint32_t e = before + incl - c;
                uint64_t m = m_me, fpos = f_me;
                while (m) {
                    if (e >= part && e < part + D8F_LIST) {
                        s_list[e - part] = c0 + (uint32_t)__builtin_ctzll(m);
                        s_pos[e - part] = fpos;
                    }
                    fpos = ~0ull;
                    ++e;
                    m &= m - 1;
                }
            }
            __syncthreads();
            const uint32_t cnt = min(total - part, (uint32_t)D8F_LIST), nrounds = (cnt + 63) / 64;
            auto chunk_of = [&](uint32_t r) -> uint32_t {
                return r < nrounds && r * 64 + (uint32_t)lane < cnt ? s_list[r * 64 + lane] : ~0u;
            };
            // a chunk's start: from the list when it is its group's first flagged chunk, else
            // gathered from fix_pos (always a load: of line 0 when not needed, no branch)
            auto pos_of = [&](uint32_t r, uint32_t ch) -> uint64_t {
                const uint64_t p = r < nrounds && r * 64 + (uint32_t)lane < cnt ? s_pos[r * 64 + lane] : 0ull;
                const uint64_t q = fix_pos[(p == ~0ull && ch != ~0u) ? ch : 0u];
                return p == ~0ull ? q : p;
            };
            uint32_t ra = (uint32_t)wv;   // round of A; B and C follow by the stride
            uint32_t cha = chunk_of(ra), chb = chunk_of(ra + D8F_WAVES);
            uint64_t posa = pos_of(ra, cha);
            uint64_t posb = pos_of(ra + D8F_WAVES, chb);
            uint4 sv[D8F_ROW / 4];
            if (ra < nrounds) load_row(sv, row_base(posa));
            while (ra < nrounds) {
                // stage round A's spans, then start round B's spans and round C's positions
                const uint64_t a0 = row_base(posa);
                put_row(sv);
                load_row(sv, row_base(posb));
                const uint32_t chc = chunk_of(ra + 2 * D8F_WAVES);
                const uint64_t posc = pos_of(ra + 2 * D8F_WAVES, chc);
                // decode round A (the clamp keeps a corrupt mask from writing past the output)
                const bool valid = cha != ~0u && (uint64_t)cha * S < n;
                const uint64_t s0 = (uint64_t)(valid ? cha : 0u) * S;
                const uint32_t cntc = valid ? (uint32_t)((n - s0 < S) ? n - s0 : S) : 0u;
                // the lane's window: row words wa, wa + 1, wa + 2 in registers, bit sh of the first;
                // a symbol reads only the table (r2 read two row words per symbol, a second LDS
                // round trip on its chain); the word after moves in when a code crosses a word
                const uint32_t cb0 = (uint32_t)(posa - (a0 << 5));
                uint32_t wa = cb0 >> 5, sh = cb0 & 31u;
                uint64_t rb = a0;   // word of `in` at row word 0
                // 4 codes move the window <= 4 words (reads up to row word wa + 6): re-stage the
                // row further on when it runs short (the window registers stay valid)
                auto restage = [&]() {
                    const uint32_t adv = wa & ~3u;
                    rb += adv;
                    wa -= adv;
                    const uint64_t nq = rb < nwords ? (nwords - rb) / 4 : 0ull;
#pragma unroll 1
                    for (int k = 0; k < D8F_ROW / 4; ++k) {   // rolled: no second set of row registers
                        const uint4 v = (uint64_t)k < nq ? reinterpret_cast<const uint4 *>(in + rb)[k] : make_uint4(0u, 0u, 0u, 0u);
                        row[4 * k] = brev8(v.x);
                        row[4 * k + 1] = brev8(v.y);
                        row[4 * k + 2] = brev8(v.z);
                        row[4 * k + 3] = brev8(v.w);
                    }
                };
                if (wa >= D8F_ROW - 6) restage();   // (a row clamped at the buffer's end)
                uint32_t w0 = row[wa], w1 = row[wa + 1], w2 = row[wa + 2];
                uint4 *const o128 = reinterpret_cast<uint4 *>(out + s0);
                uint32_t ex = 0;   // symbols >= 0x80 (gexp)
                for (uint32_t p = 0; p < (cntc + 15) / 16; ++p) {
                    uint32_t ov[4];
#pragma unroll
                    for (int q4 = 0; q4 < 4; ++q4) {
                        const uint32_t q = 4 * p + q4;
                        if (wa >= D8F_ROW - 6) restage();
                        uint32_t ob = 0;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const uint32_t lo = __builtin_amdgcn_alignbit(w1, w0, sh);
                            uint32_t e = F.lut[lo & ((1u << D8F_LUT_BITS) - 1)];
                            if (__builtin_amdgcn_ballot_w64((e & 255u) == 0u)) {   // the second level, only when a lane needs it
                                const uint32_t i2 = min(((e >> 8) << K2) | ((lo >> DC_LUT_BITS) & kmask), (uint32_t)DC_LUT2_CAP - 1);
                                const uint32_t e2 = F.lut2[(e & 255u) ? 0u : i2];
                                e = (e & 255u) ? e : e2;
                            }
                            if (e == 0) {   // past the second level (rare): canonical search
                                e = d8_long_lds(lo, __builtin_amdgcn_alignbit(w2, w1, sh), F, nary, w, pow2);
                                // the stream's partial last chunk decodes past its end: no error there
                                bad |= (e == 0 && 4 * q + k < cntc);
                            }
                            ob |= ((e >> 8) & 255u) << (8 * k);
                            sh += e & 255u;   // <= 32 bits: at most one word on
                            if (sh >= 32u) {
                                sh -= 32u;
                                w0 = w1;
                                w1 = w2;
                                w2 = row[wa + 3];
                                ++wa;
                            }
                        }
                        ov[q4] = ob;
                    }
                    if (16 * p + 16 <= cntc) o128[p] = make_uint4(ov[0], ov[1], ov[2], ov[3]);
                    else   // the stream's partial last chunk
                        for (uint32_t k = 0; 16 * p + k < cntc; ++k) out[s0 + 16 * p + k] = (uint8_t)(ov[k >> 2] >> (8 * (k & 3)));
                    if (gexp) {
#pragma unroll
                        for (int q4 = 0; q4 < 4; ++q4) {
                            const int rem = (int)cntc - (int)(16 * p) - 4 * q4;   // bytes of ov[q4] inside the chunk
                            const uint32_t keep = rem <= 0 ? 0u : rem >= 4 ? ~0u : ~(~0u << (8 * rem));
                            ex += (uint32_t)__popc(ov[q4] & keep & 0x80808080u);
                        }
                    }
                }
                if (gexp && valid) atomicAdd(gexp + cha / DC_SYNC_GROUP, ex);
                ra += D8F_WAVES;
                cha = chb; posa = posb;
                chb = chc; posb = posc;
            }
            __syncthreads();   // the list is rewritten by the next part or window
        }
    }
    if (bad) atomicOr(err, 1);
}

// base64url rendering of a bit range (int2digit alphabet, n_ary_huffman.c:371-378)
__global__ void k_base64url(const uint32_t *__restrict__ words, uint64_t bit_base, uint64_t bits,
                            char *__restrict__ text)
{
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nchar = (bits + 5) / 6;
    if (c >= nchar) return;
    const char tbl[65] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
    const uint64_t rel0 = (bit_base & 31) + c * 6;
    const uint64_t wi = rel0 >> 5;
    const uint64_t pair = ((uint64_t)bswap32(words[wi]) << 32) |
                          (((rel0 & 31) > 26) ? bswap32(words[wi + 1]) : 0u);
    uint32_t v = (uint32_t)((pair << (rel0 & 31)) >> 58);
    const uint64_t valid = bits - c * 6;
    if (valid < 6) v &= (0x3Fu << (6 - valid)) & 0x3Fu;
    text[c] = tbl[v];
}

// ------------------------------------------------------------------------------------
// Digit text of a bit range, and its inverse (the reference's intent:
// n_ary_huffman.c:46-78 "base64url / base16 / base3 / base9 ... digits", int2digit /
// digit2int :371-455, the Z85 table :389-407 for 2 base-9 or 4 base-3 digits per char, and
// "5 trits per octet, 1..243" :745-748). One character per b-bit field, MSB-first:
//   DC_TEXT_BASE64URL b=6 | DC_TEXT_BASE16 b=4 | DC_TEXT_DIGITS b=w (one base-n digit) |
//   DC_TEXT_Z85 b=8 (n=3: 4 trits, n=9: 2 digits) | DC_TEXT_TRITS5 b=10 (n=3, byte 1..243)
// A field holding a digit >= n (never written by the encoder) renders as '~' (byte 0 in
// TRITS5), which the parser rejects. Restated on the CPU by orc_text / orc_text_parse.
// ------------------------------------------------------------------------------------
__constant__ char c_b64[65] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
__constant__ char c_hex[17] = "0123456789ABCDEF";
__constant__ char c_dig[17] = "0123456789abcdef";
__constant__ char c_z85[86] = "0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ.-:+=^!/*?&<>()[]{}@%$#";

static __host__ __device__ int text_bits(int format, int n)
{
    int w = 0;
    while ((1 << w) < n) ++w;
    switch (format) {
    case DC_TEXT_BASE64URL: return 6;
    case DC_TEXT_BASE16: return 4;
    case DC_TEXT_DIGITS: return (n >= 2 && n <= 16) ? w : 0;
    case DC_TEXT_Z85: return (n == 3 || n == 9) ? 8 : 0;
    case DC_TEXT_TRITS5: return n == 3 ? 10 : 0;
    default: return 0;
    }
}

// the digits of a field (dw bits each, MSB-first) as one base-n number; -1 if one is >= n
static __device__ __forceinline__ int text_digits_value(uint32_t f, int nd, int dw, int n)
{
    int v = 0;
    for (int k = nd - 1; k >= 0; --k) {
        const int d = (int)((f >> (k * dw)) & ((1u << dw) - 1));
        if (d >= n) return -1;
        v = v * n + d;
    }
    return v;
}

__global__ void k_text(const uint32_t *__restrict__ words, uint64_t bit_base, uint64_t bits, int format, int n,
                       int b, char *__restrict__ text)
{
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nchar = (bits + b - 1) / b;
    if (c >= nchar) return;
    const uint64_t rel0 = (bit_base & 31) + c * b;
    const uint64_t wi = rel0 >> 5;   // d_words holds the word of bit_base first (as pack writes it)
    const uint32_t sh = (uint32_t)(rel0 & 31);
    const uint64_t valid = bits - c * b;   // >= 1
    const uint32_t need = valid < (uint64_t)b ? (uint32_t)valid : (uint32_t)b;   // never read past the range
    const uint64_t pair = ((uint64_t)bswap32(words[wi]) << 32) | ((sh + need > 32) ? bswap32(words[wi + 1]) : 0u);
    uint32_t f = (uint32_t)((pair << sh) >> (64 - b));
    if (valid < (uint64_t)b) f &= ~((1u << (b - valid)) - 1);
    int ch;
    switch (format) {
    case DC_TEXT_BASE64URL: ch = c_b64[f]; break;
    case DC_TEXT_BASE16: ch = c_hex[f]; break;
    case DC_TEXT_DIGITS: ch = (int)f < n ? c_dig[f] : '~'; break;
    case DC_TEXT_Z85: {
        const int v = n == 3 ? text_digits_value(f, 4, 2, 3) : text_digits_value(f, 2, 4, 9);
        ch = v < 0 ? '~' : c_z85[v];
        break;
    }
    default: {   // DC_TEXT_TRITS5
        const int v = text_digits_value(f, 5, 2, 3);
        ch = v < 0 ? 0 : 1 + v;
    }
    }
    text[c] = (char)ch;
}

// character -> field (or -1), per workgroup in LDS
static __device__ int text_field(int ch, int format, int n)
{
    switch (format) {
    case DC_TEXT_BASE64URL:
        if (ch >= 'A' && ch <= 'Z') return ch - 'A';
        if (ch >= 'a' && ch <= 'z') return ch - 'a' + 26;
        if (ch >= '0' && ch <= '9') return ch - '0' + 52;
        if (ch == '-' || ch == '+') return 62;   // digit2int takes both sets, n_ary_huffman.c:443-446
        if (ch == '_' || ch == '/') return 63;
        return -1;
    case DC_TEXT_BASE16:
    case DC_TEXT_DIGITS: {
        int d = -1;
        if (ch >= '0' && ch <= '9') d = ch - '0';
        else if (ch >= 'a' && ch <= 'f') d = ch - 'a' + 10;
        else if (format == DC_TEXT_BASE16 && ch >= 'A' && ch <= 'F') d = ch - 'A' + 10;
        return (format == DC_TEXT_DIGITS && d >= n) ? -1 : d;
    }
    case DC_TEXT_Z85: {
        int v = -1;
        for (int i = 0; i < 81; ++i)
            if (c_z85[i] == ch) v = i;
        if (v < 0) return -1;
        return n == 3 ? ((v / 27) << 6) | ((v / 9 % 3) << 4) | ((v / 3 % 3) << 2) | (v % 3) : ((v / 9) << 4) | (v % 9);
    }
    default: {   // DC_TEXT_TRITS5
        if (ch < 1 || ch > 243) return -1;
        int v = ch - 1, f = 0;
        for (int k = 0; k < 5; ++k) {
            f |= (v % 3) << (2 * k);
            v /= 3;
        }
        return f;
    }
    }
}

// one output word per thread from the <= 33 characters that cover it; bits past `bits` 0
__global__ __launch_bounds__(256) void k_text_parse(const uint8_t *__restrict__ text, uint64_t nchar, int format, int n,
                                                    int b, uint64_t bits, uint32_t *__restrict__ words,
                                                    int *__restrict__ err)
{
    __shared__ int16_t s_inv[256];
    s_inv[threadIdx.x] = (int16_t)text_field((int)threadIdx.x, format, n);
    __syncthreads();
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nwords = (bits + 31) / 32;
    if (j >= nwords) return;
    const uint64_t lo = 32 * j, c0 = lo / b, c1 = min((lo + 31) / b, nchar - 1);
    uint32_t acc = 0;
    int bad = 0;
    for (uint64_t c = c0; c <= c1; ++c) {
        const int f = s_inv[text[c]];
        bad |= f < 0;
        const int sh = 32 - (int)((int64_t)(c * b) - (int64_t)lo) - b;   // left shift of the field
        const uint32_t fu = (uint32_t)(f & 1023);
        acc |= sh >= 0 ? (uint32_t)((uint64_t)fu << sh) : fu >> (-sh);
    }
    const uint64_t valid = bits - lo;   // >= 1
    if (valid < 32) acc &= ~(0xFFFFFFFFu >> valid);
    words[j] = bswap32(acc);
    if (bad) atomicOr(err, 1);
}

// ------------------------------------------------------------------------------------
// Byte-stream codecs with a 2-state transducer: nybble static encode/decode
// (nybble_compression.c:734-1038 with modify=false) and the small front-end
// (small_compression.c:582-665) plus its inverse. Each element (input byte) maps the
// state s in {0,1} to a next state and an output byte count; composition is associative,
// so tiles of 4096 elements are summarised, scanned, and re-walked to write.
//   nybble encode, state = "a hit nybble is pending" (nybble_offset, :908-996):
//       hit : s -> 1-s, emits s bytes ; miss : s -> 0, emits 1+s bytes ; tail: +s
//   nybble decode, state = "start at the low nybble" (nybble_offset, :753-795)
//   small encode / decode: stateless counts
// ------------------------------------------------------------------------------------
// Shard bodies of the small front-end (dist.ShardedSmall): no header, no
// LITERAL fallback (decided over all ranks). BODY0: element j = byte j+1 of the stream
// (rank 0; its byte 0 is the raw first byte); BODY1: element j = byte j+1 of a shard whose
// byte 0 is the previous shard's last byte (the 1-byte left halo); both read one byte of
// right halo for a pair that starts on the shard's last byte. DBODY: decode of a body,
// element j = byte j.
// Nybble encode (M_NYB_ENC) is driven by a per-element rank: the static dictionary rank
// (c_static_rank) or, when FsmAux.rk is set, the adaptive move-to-front rank computed by the
// k_mtf_* pipeline below. The same mode writes a whole stream (FsmAux.whole: header + LITERAL
// fallback) or a shard body (dist.ShardedNybble: entry state s_init, the rank of a pending
// byte carried from the previous shard, odd-tail byte only on the last shard). M_NYB_DBODY is
// the static decode of a shard of the compressed stream (no header; one byte of right halo).
enum { M_NYB_ENC = 0, M_NYB_DEC = 1, M_SMALL_ENC = 2, M_SMALL_DEC = 3, M_SMALL_BODY0 = 4, M_SMALL_BODY1 = 5,
       M_SMALL_DBODY = 6, M_NYB_DBODY = 7 };
template <int M> struct FsmMode {
    static constexpr bool small_enc = M == M_SMALL_ENC || M == M_SMALL_BODY0 || M == M_SMALL_BODY1;
    static constexpr bool body = M == M_SMALL_BODY0 || M == M_SMALL_BODY1 || M == M_SMALL_DBODY || M == M_NYB_DBODY;
    static constexpr bool enc = M == M_SMALL_ENC;   // header + LITERAL fallback (nybble: FsmAux.whole)
    // the write pass's name in the HIP-event timings (nybble encode and decode told apart)
    static constexpr const char *wname = M == M_NYB_ENC ? "nyb_enc_write" : M == M_NYB_DEC ? "nyb_dec_write"
                                       : M == M_NYB_DBODY ? "nyb_dbody_write" : "fsm_write";
};
struct FsmAux {
    const uint8_t *rk;    // M_NYB_ENC: rank per element (0..7, 0xFF = miss); null = static dictionary
    uint32_t pend_rank;   // M_NYB_ENC body: rank of the byte before element 0 when s_init = 1
    uint32_t s_init;      // entry state of element 0
    uint32_t is_last;     // M_NYB_ENC: the shard ends the stream (odd-tail byte, :1000-1009)
    uint32_t whole;       // M_NYB_ENC: whole stream (header 0xAF x[0], LITERAL fallback)
    uint32_t tokens;      // M_NYB_DEC: a hit writes 0x80 | rank, not its static byte (k_nyb_resolve)
    // M_NYB_ENC with rk: each tile's step records (k_mtf_walk<2>, 2 uint4 each, 128 per tile),
    // whose second uint4 k_mtf_resolve made the settled ranks of the step's first touches (rk
    // holds 0xFE there, but for a tile's last element)
    const uint4 *frec;
    const uint2 *fhead;   // per tile: x = its records
};
#define FSM_SUB 1                          /* 4096-element chunks per tile */
#define FSM_TILE (4096 * FSM_SUB)

struct Fsm {
    uint32_t c0, c1;   // bytes emitted when entering in state 0 / 1
    uint32_t s0, s1;   // exit state when entering in state 0 / 1
};
static __device__ __forceinline__ Fsm fsm_id() { Fsm f; f.c0 = 0; f.c1 = 0; f.s0 = 0; f.s1 = 1; return f; }
static __device__ __forceinline__ Fsm fsm_then(const Fsm &a, const Fsm &b)
{
    Fsm r;
    r.c0 = a.c0 + (a.s0 ? b.c1 : b.c0);
    r.s0 = a.s0 ? b.s1 : b.s0;
    r.c1 = a.c1 + (a.s1 ? b.c1 : b.c0);
    r.s1 = a.s1 ? b.s1 : b.s0;
    return r;
}

// inclusive scan of compositions across a wave (lane order = element order): shuffles, no
// barrier (the 8-round Hillis-Steele over the workgroup cost 16 barriers per 4096-element tile)
static __device__ __forceinline__ Fsm fsm_wave_scan_incl(Fsm f, int lane)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        Fsm p;
        p.c0 = (uint32_t)__shfl_up((int)f.c0, d, 64);
        p.c1 = (uint32_t)__shfl_up((int)f.c1, d, 64);
        const uint32_t ss = (uint32_t)__shfl_up((int)(f.s0 | (f.s1 << 1)), d, 64);
        p.s0 = ss & 1u;
        p.s1 = ss >> 1;
        if (lane >= d) f = fsm_then(p, f);
    }
    return f;
}
static __device__ __forceinline__ uint4 fsm_pack(const Fsm &f) { return make_uint4(f.c0, f.c1, f.s0, f.s1); }

// A composition in 32 bits (counts < 2^15: a 4096-element tile emits <= 8192 bytes): half h =
// bytes emitted entering in state h | the exit state << 15. Composition: each half of a picks
// b's half by its exit state (one v_perm) and adds its count (no carry between the halves).
#define FSMP_ID 0x80000000u
static __device__ __forceinline__ uint32_t fsmp(const Fsm &f) { return f.c0 | (f.s0 << 15) | (f.c1 << 16) | (f.s1 << 31); }
static __device__ __forceinline__ Fsm fsmp_unpack(uint32_t x)
{
    Fsm f;
    f.c0 = x & 0x7FFFu; f.s0 = (x >> 15) & 1u; f.c1 = (x >> 16) & 0x7FFFu; f.s1 = x >> 31;
    return f;
}
static __device__ __forceinline__ uint32_t fsmp_then(uint32_t a, uint32_t b)
{
    const uint32_t sel = 0x01000100u + ((a >> 15) & 0x00010001u) * 0x0202u;
    return (a & 0x7FFF7FFFu) + __builtin_amdgcn_perm(b, b, sel);
}
// DPP source of a scan step (a lane with no source, or a row outside row_mask, reads FSMP_ID);
// a statement of its own (inside `?:` it ran in a branch with lanes off)
template <int CTRL, int ROWS>
static __device__ __forceinline__ uint32_t fsmp_dpp(uint32_t x)
{
    uint32_t r = (uint32_t)__builtin_amdgcn_update_dpp((int)FSMP_ID, (int)x, CTRL, ROWS, 0xf, false);
    asm volatile("" : "+v"(r));
    return r;
}
// inclusive scan across the wave (every lane active): row_shr 1, 2, 4, 8 within rows of 16,
// then row_bcast 15 and 31 (register-only: the ds_bpermute scan of fsm_wave_scan_incl issues
// 18 LDS shuffles); *ex = the exclusive value (wave_shr 1)
static __device__ __forceinline__ uint32_t fsmp_wave_scan(uint32_t f, uint32_t *ex)
{
    f = fsmp_then(fsmp_dpp<0x111, 0xf>(f), f);
    f = fsmp_then(fsmp_dpp<0x112, 0xf>(f), f);
    f = fsmp_then(fsmp_dpp<0x114, 0xf>(f), f);
    f = fsmp_then(fsmp_dpp<0x118, 0xf>(f), f);
    f = fsmp_then(fsmp_dpp<0x142, 0xa>(f), f);
    f = fsmp_then(fsmp_dpp<0x143, 0xc>(f), f);
    *ex = fsmp_dpp<0x138, 0xf>(f);
    return f;
}
static __device__ __forceinline__ Fsm fsm_unpack(const uint4 &v) { Fsm f; f.c0 = v.x; f.c1 = v.y; f.s0 = v.z; f.s1 = v.w; return f; }

__constant__ uint8_t c_static_rank[256];   // " etaoins" -> 0..7, else 0xFF (initialize_dictionary)

static __device__ __forceinline__ bool is_lower(uint32_t b) { return b >= 'a' && b <= 'z'; }

// The static dictionary " etaoins" (initialize_dictionary, nybble_compression.c:540-563) as the
// bytes of one u64, entry k in byte k: the rank of x is the position of the zero byte of
// dict ^ (x * 0x01..01) (the lowest flagged byte of the SWAR zero test is exact), 0xFF when
// absent. (A __constant__ byte table cost one divergent load per element.)
#define NYB_DICT 0x736e696f61746520ull
static __device__ __forceinline__ uint32_t static_rank(uint32_t x)
{
    constexpr uint64_t ones = 0x0101010101010101ull;
    const uint64_t t = NYB_DICT ^ (ones * (uint64_t)x);
    const uint64_t z = (t - ones) & ~t & (ones << 7);
    return z ? (uint32_t)__builtin_ctzll(z) >> 3 : 0xFFu;
}

// A lane's 16 elements read their bytes from one window of 20 bytes: window byte r = stream
// byte g0 - 1 + r, g0 = the byte of the lane's first element (element j <-> byte j + FSM_OFF).
// Lanes' windows start 16 bytes apart, so the misalignment m of the window start is the same
// in every lane: each lane loads the one aligned 16-B granule its window starts in, takes the
// next granule from the lane above (ds_bpermute; lane 63 loads its own), and five
// v_alignbyte by m cut the 20 bytes (six dword loads per lane before: 6x the address work).
// Granules wholly outside [in, in + len) are not read (zero); bytes outside it inside a read
// granule are never used by the element rules.
template <int M> struct FsmOff {
    static constexpr int v = (M == M_NYB_DEC || M == M_SMALL_DEC) ? 2 : (FsmMode<M>::body && !FsmMode<M>::small_enc) ? 0 : 1;
};
struct FsmWin {
    uint32_t w[5];
    __device__ __forceinline__ uint32_t b(int r) const { return (w[r >> 2] >> (8 * (r & 3))) & 255u; }
};
static __device__ __forceinline__ uint4 fsm_granule(uintptr_t ad, uintptr_t lo, uintptr_t hi)
{
    return (ad + 16 > lo && ad < hi) ? ld_nt(reinterpret_cast<const uint4 *>(ad)) : make_uint4(0u, 0u, 0u, 0u);
}
static __device__ __forceinline__ uint4 fsm_shfl_down1(const uint4 &v)   // lane l <- lane l + 1 (DPP; lane 63: 0)
{
    const uint32_t x = dpp_wave_shl1(v.x), y = dpp_wave_shl1(v.y), z = dpp_wave_shl1(v.z), w = dpp_wave_shl1(v.w);
    return make_uint4(x, y, z, w);
}
// every lane of the wave must call this (shuffles), also lanes without elements
static __device__ __forceinline__ FsmWin fsm_window(const uint8_t *__restrict__ in, uint64_t len, int64_t g0)
{
    const uintptr_t lo = (uintptr_t)in, hi = (uintptr_t)(in + len);
    const uintptr_t s = (uintptr_t)(in + g0 - 1);
    const uintptr_t a = s & ~(uintptr_t)15;
    const uint32_t m = (uint32_t)(s & 3), dq = (uint32_t)((s >> 2) & 3);   // byte and dword shift (uniform)
    const int lane = (int)(threadIdx.x & 63);
    const uint4 v0 = fsm_granule(a, lo, hi);
    const uint4 s1 = fsm_shfl_down1(v0);
    uint4 v1 = s1, v2 = make_uint4(0u, 0u, 0u, 0u);
    if (lane == 63) v1 = fsm_granule(a + 16, lo, hi);
    if (4 * dq + m > 14) {   // the window's 18 used bytes reach a third granule (uniform branch)
        v2 = fsm_shfl_down1(s1);   // (lane 62's is lane 63's v0 via a 0: reloaded below)
        if (lane >= 62) v2 = fsm_granule(a + 32, lo, hi);
    }
    const uint32_t d12[12] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, v2.z, v2.w};
    uint32_t d[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {   // dwords dq + q (dq uniform: selects, no register indexing)
        uint32_t v = d12[q];
#pragma unroll
        for (int k = 1; k < 4; ++k) v = dq == (uint32_t)k ? d12[q + k] : v;
        d[q] = v;
    }
    FsmWin f;
#pragma unroll
    for (int q = 0; q < 5; ++q) f.w[q] = __builtin_amdgcn_alignbyte(d[q + 1], d[q], m);
    return f;
}

// element j (lane-local k: window bytes prev = b(k), cur = b(k+1), next = b(k+2)) of mode M
template <int M>
static __device__ __forceinline__ Fsm elem_fsm(const FsmWin &W, int k, uint64_t len, uint64_t j, uint32_t rk)
{
    Fsm f;
    const uint32_t x = W.b(k + 1);
    if (M == M_NYB_ENC) {                // byte i = j+1; rk = its rank (0xFF = miss)
        if (rk != 0xFF) { f.c0 = 0; f.c1 = 1; f.s0 = 1; f.s1 = 0; }
        else { f.c0 = 1; f.c1 = 2; f.s0 = 0; f.s1 = 0; }
    } else if (M == M_NYB_DEC || M == M_NYB_DBODY) {   // compressed byte k = j+2 (a body: byte j)
        const uint32_t h = x >> 4, l = x & 15;
        if (h & 8) { f.c0 = 2; f.s0 = (l & 8) ? 0 : 1; }
        else { f.c0 = 1; f.s0 = 0; }
        f.c1 = 1;
        f.s1 = (l & 8) ? 0 : 1;
    } else if (FsmMode<M>::small_enc) {   // byte i = j+1
        const uint64_t i = j + 1;
        const bool second = (M == M_SMALL_BODY1 || i >= 2) && W.b(k) == ' ' && is_lower(x);
        f.c0 = f.c1 = second ? 0 : 1;
        f.s0 = f.s1 = 0;
    } else {                             // small decode, byte k = j+2 (a body: byte j)
        f.c0 = f.c1 = (x >= 0x80) ? 2 : 1;
        f.s0 = f.s1 = 0;
    }
    (void)len;
    return f;
}

// the lane's 16 ranks (adaptive nybble: aux.rk, element-indexed and 16-B aligned at j0), or
// the static dictionary's ranks of the window bytes
// the static ranks in LDS (one byte per value, filled by the workgroup: fsm_rank_table):
// random reads of 64 dwords, mostly broadcasts on text (the SWAR search of the dictionary, a
// 64-bit multiply and zero test per element, made the tile count kernel VALU-bound: 0.68 ->
// 0.94 ms per GiB)
// The kernels' small lookup tables, built at compile time (built per workgroup they cost ~90
// VALU in every wave of the nybble writer: ~12% of its instructions)
struct NybTables {
    uint32_t rank4[64];              // static ranks, 4 bytes per dword
    uint32_t esel_lo[256], esel_hi[256];   // k_fsm_write's v_perm selectors, per 8-bit pattern
    uint32_t dsel_lo[16], dsel_hi[16];     // k_small_write's (decode), per 4-bit pair pattern
    constexpr NybTables() : rank4(), esel_lo(), esel_hi(), dsel_lo(), dsel_hi()
    {
        const char dict[9] = " etaoins";
        for (int x = 0; x < 256; ++x) {
            uint32_t r = 0xFFu;
            for (int k = 7; k >= 0; --k) if ((uint8_t)dict[k] == x) r = (uint32_t)k;
            rank4[x >> 2] |= r << (8 * (x & 3));
        }
        // pattern t = c1 | c2 << 4 (bit i: element i writes its first / its second byte): the
        // output bytes in order, first byte i = selector i (S1 = the first bytes), second byte
        // i = selector 4 + i (S0 = the second bytes); 0x0c = a zero byte
        for (int t = 0; t < 256; ++t) {
            uint32_t sel[2] = {0x0c0c0c0cu, 0x0c0c0c0cu};
            int o = 0;
            for (int i = 0; i < 4; ++i) {
                if ((t >> i) & 1) { sel[o >> 2] = (sel[o >> 2] & ~(255u << (8 * (o & 3)))) | ((uint32_t)i << (8 * (o & 3))); ++o; }
                if ((t >> (4 + i)) & 1) {
                    sel[o >> 2] = (sel[o >> 2] & ~(255u << (8 * (o & 3)))) | ((uint32_t)(4 + i) << (8 * (o & 3)));
                    ++o;
                }
            }
            esel_lo[t] = sel[0];
            esel_hi[t] = sel[1];
        }
        // pattern t (bit i: byte i >= 0x80): byte i -> ' ' (S1) then byte i & 0x7F (S0), else
        // byte i (S0); 0x0c = a zero byte
        for (int t = 0; t < 16; ++t) {
            uint32_t sel[2] = {0x0c0c0c0cu, 0x0c0c0c0cu};
            int o = 0;
            for (int i = 0; i < 4; ++i) {
                if ((t >> i) & 1) { sel[o >> 2] = (sel[o >> 2] & ~(255u << (8 * (o & 3)))); ++o; }
                sel[o >> 2] = (sel[o >> 2] & ~(255u << (8 * (o & 3)))) | ((uint32_t)(4 + i) << (8 * (o & 3)));
                ++o;
            }
            dsel_lo[t] = sel[0];
            dsel_hi[t] = sel[1];
        }
    }
};
__constant__ NybTables c_nyb = NybTables();

static __device__ __forceinline__ void fsm_rank_table(uint8_t *s_rank)
{
    if (threadIdx.x < 64) reinterpret_cast<uint32_t *>(s_rank)[threadIdx.x] = c_nyb.rank4[threadIdx.x];
}
template <int M>
static __device__ __forceinline__ void fsm_ranks(const FsmWin &W, const FsmAux &aux, uint64_t j0, uint64_t nelem,
                                                 uint32_t (&rk)[16], const uint8_t *s_rank,
                                                 const uint4 *pP = nullptr, const uint4 *pre = nullptr)
{
    if (M != M_NYB_ENC) return;
    if (aux.rk) {
        uint4 v = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        if (j0 + 16 <= nelem) v = pre ? *pre : *reinterpret_cast<const uint4 *>(aux.rk + j0);   // (pre: loaded early)
        else for (uint64_t q = 0; j0 + q < nelem; ++q) {
            const uint32_t r = aux.rk[j0 + q];
            const uint32_t sh = 8 * (q & 3), msk = ~(255u << sh);
            if (q < 4) v.x = (v.x & msk) | (r << sh); else if (q < 8) v.y = (v.y & msk) | (r << sh);
            else if (q < 12) v.z = (v.z & msk) | (r << sh); else v.w = (v.w & msk) | (r << sh);
        }
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; ++k) rk[k] = (w4[k >> 2] >> (8 * (k & 3))) & 255u;
        if (pP) {   // first touches (0xFE): the settled ranks of the lane's step record (LDS)
            const uint4 P = *pP;
            const uint32_t p4[4] = {P.x, P.y, P.z, P.w};
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (rk[k] == 0xFEu) rk[k] = (p4[k >> 2] >> (8 * (k & 3))) & 255u;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) rk[k] = s_rank[W.b(k + 1)];
    }
}

// ---- the nybble transducers' states, 16 elements at once (bit k = element k of a lane) ----
// Both machines are two-state, and a lane's 16 states follow from its element flags by one
// 32-bit add: a carry is generated where an element forces state 1, killed where it forces 0
// and propagated where the state carries over, so with A = generate | propagate and
// B = generate, A + B + s0 carries c_{k-1} = (sum ^ propagate) bit k into element k, which is
// its state s_k (bit 16: the state after the lane). (r2 composed the 16 elements' transition
// functions one after another: ~30 VALU per element in the count pass, ~74 in the writer.)
// bit `bit` of the lane's window bytes 1..16 (element k = window byte k + 1)
static __device__ __forceinline__ uint32_t fsm_byte_bits(const FsmWin &W, int bit)
{
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t X = __builtin_amdgcn_alignbyte(W.w[q + 1], W.w[q], 1);   // bytes 4q+1..4q+4
        uint32_t b = (X >> bit) & 0x01010101u;
        b = (b | (b >> 7) | (b >> 14) | (b >> 21)) & 15u;
        m |= b << (4 * q);
    }
    return m;
}
// the states from s0, bit k = s_k (k <= 16); g, p: generate and propagate masks (disjoint)
static __device__ __forceinline__ uint32_t fsm_carry_states(uint32_t g, uint32_t p, uint32_t s0)
{
    return ((g | p) + g + s0) ^ p;
}
// decode (s = "at the low nybble"): s' = (s | h) & !l, h / l = bits 7 / 3 of the byte;
// elements outside `valid` keep the state. Returns the states (bits 0..16).
static __device__ __forceinline__ uint32_t nyb_dec_states(uint32_t H, uint32_t L, uint32_t valid, uint32_t s0)
{
    const uint32_t g = H & ~L & valid, p = (~H & ~L & valid) | (~valid & 0xFFFFu);
    return fsm_carry_states(g, p, s0);
}
// encode (s = "a hit nybble is pending"): a hit toggles the state, a miss clears it. With P_k
// the parity of the hits before k, s_k = P_k ^ (P at the last miss before k, or s0): the value
// at the last miss is carried forward through the hits (a carry generated at a miss where
// P = 1, killed at one where P = 0). Returns the states (bits 0..16).
static __device__ __forceinline__ uint32_t nyb_enc_states(uint32_t Hm, uint32_t valid, uint32_t s0)
{
    Hm &= valid;       // (window bytes past the stream may read as hits)
    uint32_t X = Hm;   // inclusive prefix parity
    X ^= X << 1;
    X ^= X << 2;
    X ^= X << 4;
    X ^= X << 8;
    const uint32_t P = (X << 1) & 0x1FFFFu;   // exclusive: bit k = parity of hits before k
    const uint32_t miss = ~Hm & valid;
    const uint32_t g = miss & P, p = Hm | (~valid & 0xFFFFu);
    return (P ^ fsm_carry_states(g, p, s0)) & 0x1FFFFu;
}
// the lane's composition (both entry states): counts and exit states
template <int M>
static __device__ __forceinline__ Fsm nyb_lane_fsm(uint32_t A, uint32_t B, uint32_t valid)
{
    Fsm f;
    if (M == M_NYB_ENC) {   // A = hit mask
        A &= valid;
        const uint32_t miss = ~A & valid;
        const uint32_t S0 = nyb_enc_states(A, valid, 0u), S1 = nyb_enc_states(A, valid, 1u);
        f.c0 = __popc(A & S0 & 0xFFFFu) + __popc(miss) + __popc(miss & S0);
        f.c1 = __popc(A & S1 & 0xFFFFu) + __popc(miss) + __popc(miss & S1);
        f.s0 = (S0 >> 16) & 1u;
        f.s1 = (S1 >> 16) & 1u;
    } else {                // A = high-nybble flags, B = low-nybble flags
        const uint32_t S0 = nyb_dec_states(A, B, valid, 0u), S1 = nyb_dec_states(A, B, valid, 1u);
        f.c0 = __popc(valid) + __popc(valid & A & ~S0);
        f.c1 = __popc(valid) + __popc(valid & A & ~S1);
        f.s0 = (S0 >> 16) & 1u;
        f.s1 = (S1 >> 16) & 1u;
    }
    return f;
}
// the lane's flag masks: encode, the hit mask of its ranks; decode, bits 7 and 3 of its bytes
template <int M>
static __device__ __forceinline__ void nyb_lane_flags(const FsmWin &W, const uint32_t (&rk)[16], uint32_t &A, uint32_t &B)
{
    if (M == M_NYB_ENC) {
        A = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) A |= (rk[k] != 0xFFu ? 1u : 0u) << k;
        B = 0;
    } else {
        A = fsm_byte_bits(W, 7);
        B = fsm_byte_bits(W, 3);
    }
}

template <int M>
__global__ __launch_bounds__(256) void k_fsm_tiles(const uint8_t *__restrict__ in, uint64_t len,
                                                   uint64_t nelem, uint4 *__restrict__ summ, FsmAux aux)
{
    __shared__ uint4 s_f[FSM_SUB][4];   // wave totals per chunk
    __shared__ __attribute__((aligned(4))) uint8_t s_rank[256];
    const int t = threadIdx.x;
    if (M == M_NYB_ENC && !aux.rk) { fsm_rank_table(s_rank); __syncthreads(); }
    // chunk c of the tile: elements [c * 4096 + 16 t, +16) for lane t (coalesced per chunk);
    // all chunks' windows are loaded before any is walked
    FsmWin W[FSM_SUB];
#pragma unroll
    for (int c = 0; c < FSM_SUB; ++c)
        W[c] = fsm_window(in, len, (int64_t)((uint64_t)blockIdx.x * FSM_TILE + (uint64_t)c * 4096 + (uint64_t)t * 16) +
                                       FsmOff<M>::v);   // every lane (shuffles)
#pragma unroll
    for (int c = 0; c < FSM_SUB; ++c) {
        const uint64_t j0 = (uint64_t)blockIdx.x * FSM_TILE + (uint64_t)c * 4096 + (uint64_t)t * 16;
        Fsm f = fsm_id();
        if (j0 < nelem) {
            uint32_t rk[16], A, B;
            fsm_ranks<M>(W[c], aux, j0, nelem, rk, s_rank);
            nyb_lane_flags<M>(W[c], rk, A, B);
            const uint32_t valid = nelem - j0 >= 16 ? 0xFFFFu : (1u << (uint32_t)(nelem - j0)) - 1u;
            f = nyb_lane_fsm<M>(A, B, valid);
        }
        const Fsm inc = fsm_wave_scan_incl(f, t & 63);
        if ((t & 63) == 63) s_f[c][t >> 6] = fsm_pack(inc);
    }
    __syncthreads();
    if (t == 0) {
        Fsm a = fsm_id();
#pragma unroll
        for (int q = 0; q < 4 * FSM_SUB; ++q) a = fsm_then(a, fsm_unpack(s_f[q >> 2][q & 3]));
        summ[blockIdx.x] = fsm_pack(a);
    }
}

// The nybble transducers' tile summaries (static encode, decode, decode body), one wave per
// tile: a lane takes 64 contiguous elements as four aligned 16-B granules of the tile's bytes
// (lane 63 a fifth when the tile is not granule-aligned), folds their 16-element compositions
// (nyb_lane_fsm) and the wave scans once per tile. The element rules need only each element's
// own byte, so no neighbour window. (k_fsm_tiles: 16 elements per lane, a workgroup barrier and
// a serial fold per 4096-element tile: 0.48 ms per GiB of static encode, 0.30 of decode.)
static __device__ __forceinline__ uint32_t byte_bits4(uint32_t d, int bit)   // bit `bit` of 4 bytes
{
    uint32_t b = (d >> bit) & 0x01010101u;
    return (b | (b >> 7) | (b >> 14) | (b >> 21)) & 15u;
}
#define NYB_TPW 2   /* tiles per wave: the second tile's granules load while the first is folded */
template <int M>
__global__ __launch_bounds__(256) void k_nyb_tiles(const uint8_t *__restrict__ in, uint64_t len, uint64_t nelem,
                                                   uint64_t ntiles, uint4 *__restrict__ summ)
{
    static_assert(M == M_NYB_ENC || M == M_NYB_DEC || M == M_NYB_DBODY, "nybble transducers");
    __shared__ uint8_t s_hit[256];   // static encode: 1 for the dictionary's bytes
    const int t = threadIdx.x, lane = t & 63;
    if (M == M_NYB_ENC) {
        s_hit[t] = ((c_nyb.rank4[t >> 2] >> (8 * (t & 3))) & 255u) != 0xFFu ? 1u : 0u;
        __syncthreads();
    }
    const uint64_t Tw = ((uint64_t)blockIdx.x * 4 + (uint64_t)(t >> 6)) * NYB_TPW;
    if (Tw >= ntiles) return;   // whole waves (no barriers below)
    uint4 v[NYB_TPW][5];
    uint32_t nvs[NYB_TPW], shs[NYB_TPW];
#pragma unroll
    for (int u = 0; u < NYB_TPW; ++u) {
        const uint64_t T = Tw + u;
        const uint64_t j0 = T * FSM_TILE;
        const uint32_t nv = T >= ntiles ? 0u : nelem - j0 < FSM_TILE ? (uint32_t)(nelem - j0) : (uint32_t)FSM_TILE;
        const uint64_t B0 = j0 + FsmOff<M>::v;                                  // the tile's first byte
        const uint32_t sh = (uint32_t)((B0 + ((uintptr_t)in & 15u)) & 15u);    // its place in its granule
        const int64_t g0 = (int64_t)B0 - (int64_t)sh;                           // granule 0 (may begin before in)
        nvs[u] = nv; shs[u] = sh;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int64_t o = g0 + 16 * (4 * lane + i);
            const bool want = nv && (i < 4 || (lane == 63 && sh != 0));
            v[u][i] = (want && o < (int64_t)len) ? *reinterpret_cast<const uint4 *>(in + o) : make_uint4(0u, 0u, 0u, 0u);
        }
    }
#pragma unroll
    for (int u = 0; u < NYB_TPW; ++u) {
        if (Tw + u >= ntiles) break;   // (uniform)
        const uint32_t nv = nvs[u], sh = shs[u];
        Fsm acc = fsm_id();
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            // elements of granule gi: its bytes b with 0 <= 16 gi + b - sh < nv
            const int gi = 4 * lane + i;
            const int lo = min(max((int)sh - 16 * gi, 0), 16), hi = min(max((int)nv + (int)sh - 16 * gi, 0), 16);
            uint32_t valid = hi > lo ? (1u << hi) - (1u << lo) : 0u;
            if (i == 4 && lane != 63) valid = 0u;
            const uint32_t d[4] = {v[u][i].x, v[u][i].y, v[u][i].z, v[u][i].w};
            uint32_t A = 0, B = 0;
            if (M == M_NYB_ENC) {
#pragma unroll
                for (int k = 0; k < 16; ++k) A |= (uint32_t)s_hit[(d[k >> 2] >> (8 * (k & 3))) & 255u] << k;
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) { A |= byte_bits4(d[q], 7) << (4 * q); B |= byte_bits4(d[q], 3) << (4 * q); }
            }
            acc = fsm_then(acc, nyb_lane_fsm<M>(A, B, valid));
        }
        uint32_t xp;
        const uint32_t inc = fsmp_wave_scan(fsmp(acc), &xp);
        if (lane == 63) summ[Tw + u] = fsm_pack(fsmp_unpack(inc));
    }
}

// Scan of the tile summaries in two levels, all accesses coalesced: k_fsm_scan_up turns each
// group of 1024 tile summaries into local exclusive compositions (in place) and one group
// summary; k_fsm_scan (below) then scans the group summaries; a tile's entry is its group's
// entry followed by its local composition (k_fsm_write). (One workgroup walking 262144
// tile summaries with 4-KiB-strided lanes took 0.6 ms on 1 GiB.)
#define FSM_GROUP 1024
__global__ __launch_bounds__(FSM_GROUP) void k_fsm_scan_up(uint4 *__restrict__ summ, uint64_t ntiles,
                                                           uint4 *__restrict__ gsum)
{
    __shared__ uint4 s_f[FSM_GROUP];
    const int t = threadIdx.x;
    const uint64_t k = (uint64_t)blockIdx.x * FSM_GROUP + t;
    const uint4 mine = k < ntiles ? summ[k] : make_uint4(0u, 0u, 0u, 1u);
    s_f[t] = mine;
    __syncthreads();
    for (int d = 1; d < FSM_GROUP; d <<= 1) {
        uint4 p = make_uint4(0u, 0u, 0u, 1u);
        const bool has = t >= d;
        if (has) p = s_f[t - d];
        const uint4 me = s_f[t];
        __syncthreads();
        if (has) {
            Fsm fa, fb;
            fa.c0 = p.x; fa.c1 = p.y; fa.s0 = p.z; fa.s1 = p.w;
            fb.c0 = me.x; fb.c1 = me.y; fb.s0 = me.z; fb.s1 = me.w;
            const Fsm r = fsm_then(fa, fb);
            s_f[t] = make_uint4(r.c0, r.c1, r.s0, r.s1);
        }
        __syncthreads();
    }
    if (k < ntiles) summ[k] = t ? s_f[t - 1] : make_uint4(0u, 0u, 0u, 1u);
    if (t == FSM_GROUP - 1) gsum[blockIdx.x] = s_f[FSM_GROUP - 1];
}

// single workgroup: tile entry (offset, state) from the summaries, starting in state s_init;
// meta[0] = total count, meta[1] = final state (from s_init); meta[2..5] = the whole
// composition (c0, c1, s0, s1) for shard plans
__global__ __launch_bounds__(1024) void k_fsm_scan(const uint4 *__restrict__ summ, uint64_t ntiles,
                                                   uint64_t *__restrict__ entry, uint64_t *__restrict__ meta,
                                                   uint32_t s_init)
{
    __shared__ uint64_t s_c0[1024], s_c1[1024];
    __shared__ uint32_t s_s0[1024], s_s1[1024];
    const int t = threadIdx.x;
    const uint64_t per = (ntiles + 1023) / 1024;
    const uint64_t a0 = (uint64_t)t * per;
    const uint64_t a1 = (a0 + per < ntiles) ? a0 + per : ntiles;
    uint64_t c0 = 0, c1 = 0;
    uint32_t s0 = 0, s1 = 1;
    for (uint64_t k0 = a0; k0 < a1; k0 += 8) {   // 8 summaries in flight per lane
        uint4 bb[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) bb[q] = k0 + q < a1 ? summ[k0 + q] : make_uint4(0u, 0u, 0u, 1u);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint4 b = bb[q];
            const uint64_t n0 = c0 + (s0 ? b.y : b.x), n1 = c1 + (s1 ? b.y : b.x);
            const uint32_t m0 = s0 ? b.w : b.z, m1 = s1 ? b.w : b.z;
            c0 = n0; c1 = n1; s0 = m0; s1 = m1;
        }
    }
    s_c0[t] = c0; s_c1[t] = c1; s_s0[t] = s0; s_s1[t] = s1;
    __syncthreads();
    // inclusive Hillis-Steele over compositions (left operand = earlier)
    for (int d = 1; d < 1024; d <<= 1) {
        uint64_t pc0 = 0, pc1 = 0;
        uint32_t ps0 = 0, ps1 = 1;
        const bool has = t >= d;
        if (has) { pc0 = s_c0[t - d]; pc1 = s_c1[t - d]; ps0 = s_s0[t - d]; ps1 = s_s1[t - d]; }
        const uint64_t mc0 = s_c0[t], mc1 = s_c1[t];
        const uint32_t ms0 = s_s0[t], ms1 = s_s1[t];
        __syncthreads();
        if (has) {
            s_c0[t] = pc0 + (ps0 ? mc1 : mc0);
            s_s0[t] = ps0 ? ms1 : ms0;
            s_c1[t] = pc1 + (ps1 ? mc1 : mc0);
            s_s1[t] = ps1 ? ms1 : ms0;
        }
        __syncthreads();
    }
    // exclusive prefix applied to the initial state 0
    uint64_t off = 0;
    uint32_t st = s_init;
    if (t > 0) { off = s_init ? s_c1[t - 1] : s_c0[t - 1]; st = s_init ? s_s1[t - 1] : s_s0[t - 1]; }
    for (uint64_t k0 = a0; k0 < a1; k0 += 8) {
        uint4 bb[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) bb[q] = k0 + q < a1 ? summ[k0 + q] : make_uint4(0u, 0u, 0u, 1u);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if (k0 + q < a1) entry[k0 + q] = (off << 1) | st;
            const uint4 b = bb[q];
            off += st ? b.y : b.x;
            st = st ? b.w : b.z;
        }
    }
    if (t == 1023) {
        meta[0] = s_init ? s_c1[1023] : s_c0[1023];
        meta[1] = s_init ? s_s1[1023] : s_s0[1023];
        meta[2] = s_c0[1023]; meta[3] = s_c1[1023]; meta[4] = s_s0[1023]; meta[5] = s_s1[1023];
    }
}

// Re-walk each tile with its entry state and write the output bytes.
//   layout: nybble/small encode: out[0] = type, out[1] = x[0], body at out[2..];
//           decoders: out[0] = in[1], body at out[1..]. Encoders fall back to
//           LITERAL (' ' + raw, :1018-1037) when the stream is not shorter than n.
template <int M>
__global__ __launch_bounds__(256) void k_fsm_write(const uint8_t *__restrict__ in, uint64_t len, uint64_t nelem,
                                                   const uint64_t *__restrict__ entry, const uint4 *__restrict__ loc,
                                                   const uint64_t *__restrict__ meta, uint8_t *__restrict__ out,
                                                   FsmAux aux)
{
    static_assert(M == M_NYB_ENC || M == M_NYB_DEC || M == M_NYB_DBODY, "nybble modes (the small codec: k_small_write)");
    // the tile's output (<= 2 bytes per element) is staged in LDS, s_out[x] = out[o_al + x]
    // with o_al the 16-B granule of its first byte, then stored as whole uint4s (bytes only in
    // the two granules shared with the neighbouring tiles)
    __shared__ uint4 s_f[FSM_SUB][4];   // wave totals per chunk
    __shared__ __attribute__((aligned(16))) uint8_t s_out[2 * FSM_TILE + 32];
    __shared__ __attribute__((aligned(4))) uint8_t s_rank[256];
    __shared__ uint2 s_esel[256];   // v_perm selectors per 4-element pattern
    // adaptive encode: the tile's step records (<= 128: one per thread), by step = lane
    __shared__ uint8_t s_map[M == M_NYB_ENC ? 256 : 1];   // step -> record + 1 (0: none)
    __shared__ uint4 s_P[M == M_NYB_ENC ? 128 : 1];       // a record's settled first-touch ranks
    const int t = threadIdx.x;
    if (M == M_NYB_ENC && !aux.rk) fsm_rank_table(s_rank);
    const bool patch = M == M_NYB_ENC && aux.rk && aux.frec;
    if (patch) {
        s_map[t] = 0;
        const uint32_t nrec = aux.fhead[blockIdx.x].x;
        uint4 q0 = make_uint4(0u, 0u, 0u, 0u), q1 = q0;
        if ((uint32_t)t < nrec) {
            const uint4 *const r = aux.frec + 2 * ((uint64_t)blockIdx.x * 128 + t);
            q0 = r[0];
            q1 = r[1];
        }
        __syncthreads();
        if ((uint32_t)t < nrec) {
            s_map[q0.z & 255u] = (uint8_t)(t + 1);
            s_P[t] = q1;
        }
    }
    s_esel[t] = make_uint2(c_nyb.esel_lo[t], c_nyb.esel_hi[t]);   // (NybTables)
    const bool nyb_whole = M == M_NYB_ENC && aux.whole;
    const bool enc = FsmMode<M>::enc || nyb_whole;
    // every global read the tile needs is issued here, before the first one is waited for (the
    // LITERAL test on meta, then the window, then entry/loc after the barrier: three round trips)
    FsmWin W_[FSM_SUB];
#pragma unroll
    for (int c = 0; c < FSM_SUB; ++c)
        W_[c] = fsm_window(in, len, (int64_t)((uint64_t)blockIdx.x * FSM_TILE + (uint64_t)c * 4096 + (uint64_t)t * 16) +
                                       FsmOff<M>::v);   // every lane (shuffles)
    const uint64_t e = entry[blockIdx.x / FSM_GROUP];
    const uint4 lc = loc[blockIdx.x];
    static_assert(FSM_SUB == 1, "one chunk per tile: the lane's step is t (rkpre, s_map)");
    uint4 rkpre = make_uint4(~0u, ~0u, ~0u, ~0u);   // adaptive: the lane's 16 ranks, with the window
    {
        const uint64_t j0 = (uint64_t)blockIdx.x * FSM_TILE + (uint64_t)t * 16;   // (FSM_SUB = 1)
        if (M == M_NYB_ENC && aux.rk && j0 + 16 <= nelem) rkpre = *reinterpret_cast<const uint4 *>(aux.rk + j0);
    }
    const uint64_t body = (M == M_NYB_ENC) ? meta[0] + (aux.is_last ? meta[1] : 0) : meta[0];
    const uint64_t total = enc ? 2 + body : 1 + body;
    const bool literal = enc && total >= len;
    if (literal) {
        // copy x -> out[1..len], one grid-stride pass
        for (uint64_t i = (uint64_t)blockIdx.x * 256 + t; i < len; i += (uint64_t)gridDim.x * 256)
            out[1 + i] = in[i];
        if (blockIdx.x == 0 && t == 0) out[0] = ' ';
        return;
    }
    const bool headed = M == M_NYB_ENC ? nyb_whole : !FsmMode<M>::body;
    if (blockIdx.x == 0 && t == 0 && headed) {
        if (M == M_NYB_ENC) { out[0] = 0xAF; out[1] = in[0]; }
        else if (M == M_SMALL_ENC) { out[0] = 8; out[1] = in[0]; }
        else { out[0] = in[1]; }
    }
    for (uint32_t i = (uint32_t)t; i < (2 * FSM_TILE + 32) / 16; i += 256)   // the stage is OR-merged into
        reinterpret_cast<uint4 *>(s_out)[i] = make_uint4(0u, 0u, 0u, 0u);
    if (M == M_NYB_ENC && (!aux.rk || patch)) __syncthreads();   // s_rank, s_patch (the stage: ordered by the scan's barrier)
    // per chunk: the lane's composition, scanned across the wave (shuffles); the wave totals of
    // every chunk through LDS (one barrier)
    const int lane = t & 63, wid = t >> 6;
    Fsm ex[FSM_SUB];   // lanes before this one in the wave, per chunk
    uint32_t fa[FSM_SUB], fb[FSM_SUB], fvalid[FSM_SUB];   // the lane's element flags (nyb_lane_flags)
    uint32_t RKp[FSM_SUB][4];   // encode: the lane's 16 ranks, 4 per dword (kept for the writer)
#pragma unroll
    for (int c = 0; c < FSM_SUB; ++c) {
        const uint64_t j0 = (uint64_t)blockIdx.x * FSM_TILE + (uint64_t)c * 4096 + (uint64_t)t * 16;
        fa[c] = fb[c] = 0u;
        fvalid[c] = j0 >= nelem ? 0u : nelem - j0 >= 16 ? 0xFFFFu : (1u << (uint32_t)(nelem - j0)) - 1u;
        RKp[c][0] = RKp[c][1] = RKp[c][2] = RKp[c][3] = ~0u;
        Fsm f = fsm_id();
        if (j0 < nelem) {
            uint32_t rk[16];
            const uint32_t mr = patch ? s_map[t] : 0u;   // (FSM_SUB = 1: the lane's step is t)
            fsm_ranks<M>(W_[c], aux, j0, nelem, rk, s_rank, mr ? &s_P[M == M_NYB_ENC ? mr - 1 : 0] : nullptr, &rkpre);
            nyb_lane_flags<M>(W_[c], rk, fa[c], fb[c]);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                RKp[c][q] = (rk[4 * q] & 255u) | ((rk[4 * q + 1] & 255u) << 8) | ((rk[4 * q + 2] & 255u) << 16) |
                            ((rk[4 * q + 3] & 255u) << 24);
            f = nyb_lane_fsm<M>(fa[c], fb[c], fvalid[c]);
        }
        uint32_t xp;
        const uint32_t inc = fsmp_wave_scan(fsmp(f), &xp);
        if (lane == 63) s_f[c][wid] = fsm_pack(fsmp_unpack(inc));
        ex[c] = fsmp_unpack(xp);
    }
    __syncthreads();
    // entry = the group's entry, then the tile's local exclusive composition (k_fsm_scan_up)
    const uint32_t s_g = (uint32_t)(e & 1);
    const uint64_t o_tile = (e >> 1) + (s_g ? lc.y : lc.x) + (headed ? (enc ? 2 : 1) : 0);   // first output byte
    const uint32_t s_tile = s_g ? lc.w : lc.z;
    Fsm run = fsm_id();   // chunks before c, then waves before this one in chunk c
    uint64_t o_c[FSM_SUB];
    uint32_t st_c[FSM_SUB];
#pragma unroll
    for (int c = 0; c < FSM_SUB; ++c) {
        Fsm pre = run;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const Fsm w = fsm_unpack(s_f[c][q]);
            if (q < wid) pre = fsm_then(pre, w);
            run = fsm_then(run, w);
        }
        const Fsm x = fsm_then(pre, ex[c]);
        o_c[c] = o_tile + (s_tile ? x.c1 : x.c0);
        st_c[c] = s_tile ? x.s1 : x.s0;
    }
    const uint64_t s_end = o_tile + (s_tile ? run.c1 : run.c0);   // the tile's end
    // granule of the tile's first byte, relative to out (negative when out is unaligned and
    // the tile starts in out's first granule)
    const int64_t o_al = (int64_t)((((uintptr_t)(out + o_tile)) & ~(uintptr_t)15) - (uintptr_t)out);
    // Each lane's output is one contiguous run (its elements in order): the bytes are computed
    // branch-free per element (count 0-2, value, next state) and packed into a 64-bit
    // accumulator, whose complete dwords are OR-ed into the zeroed LDS stage (dwords shared
    // with the neighbouring lanes' runs merge without ordering). (r2 stored each byte into the
    // stage under per-element branches: 2.0 ms per GiB of nybble encode.)
    // hit table: " etaoins" as one u64, or the token bytes 0x80 | rank (aux.tokens)
    const uint64_t tblv = aux.tokens ? 0x8786858483828180ull : NYB_DICT;
    uint32_t *const s_out32 = reinterpret_cast<uint32_t *>(s_out);
#pragma unroll
    for (int c = 0; c < FSM_SUB; ++c) {
        const uint64_t j0 = (uint64_t)blockIdx.x * FSM_TILE + (uint64_t)c * 4096 + (uint64_t)t * 16;
        if (j0 >= nelem) continue;
        const FsmWin &W = W_[c];
        const uint64_t o0 = o_c[c];
        // every element's state at once, from the lane's entry state
        const uint32_t S = M == M_NYB_ENC ? nyb_enc_states(fa[c], fvalid[c], st_c[c])
                                          : nyb_dec_states(fa[c], fb[c], fvalid[c], st_c[c]);
        const uint32_t P = (uint32_t)((int64_t)o0 - o_al);   // stage byte of the lane's first output
        uint32_t di = P >> 2, nb = 8u * (P & 3u);
        uint64_t acc = 0;
        const uint32_t kend = nelem - j0 < 16 ? (uint32_t)(nelem - j0) : 16u;
        const uint32_t valid = fvalid[c];
        if (M == M_NYB_ENC) {
            // masks of the lane's elements: a hit, and the state before it; an element past the
            // input counts as a hit in state 0 (no bytes)
            const uint32_t Hx = (fa[c] & valid) | (~valid & 0xFFFFu), Sx = S & valid;
            // the rank of the pending hit before element 0: the previous window byte's, or the
            // shard's carried one
            uint32_t rp0 = j0 ? (aux.rk ? (uint32_t)aux.rk[j0 - 1] : (uint32_t)s_rank[W.b(0)]) : aux.pend_rank;
            if (patch && rp0 == 0xFEu && t > 0) {   // (lane 0: the tile's last element is settled in rk)
                const uint32_t mp = s_map[t - 1];
                if (mp) rp0 = s_P[mp - 1].w >> 24;
            }
            if (aux.is_last && len >= 2 && len - 2 >= j0 && len - 2 < j0 + kend) {
                // odd tail (:1000-1009): the stream's last element a hit left pending: its byte,
                // raw, after the bytes of the elements before it
                const uint32_t kt = (uint32_t)(len - 2 - j0);
                if (((Hx & ~Sx) >> kt) & 1u) {
                    const uint32_t below = (1u << kt) - 1u;
                    const uint32_t before = __popc(~Hx & below) + __popc(Sx & below);
                    uint32_t w = W.w[0];   // window byte kt + 1 (a runtime index: selects)
#pragma unroll
                    for (uint32_t q = 1; q < 5; ++q) w = ((kt + 1) >> 2) == q ? W.w[q] : w;
                    out[o0 + before] = (uint8_t)(w >> (8 * ((kt + 1) & 3)));
                }
            }
            // Each element writes 0-2 bytes: its first byte (a miss, or any element after a
            // pending hit) = s ? (h ? pair : prev) : x, its second (a miss after a pending hit) = x.
            // Four elements at a time in SWAR: the dword of their first bytes B1 and of their own
            // bytes X, then two v_perm place their 0-8 output bytes in order (selectors by the
            // 8-bit pattern of who writes what, s_esel), and the lane's run advances by whole
            // dwords OR-ed into the zeroed stage at its bit offset (the partial last dword too:
            // ORs are idempotent, so the pending bits are OR-ed again with the next ones).
            // ~9 VALU per element. (r4's per-element byte stores at a running offset: ~25 VALU and
            // 2 LDS byte stores per element; r3's 64-bit accumulator flushed every 2 elements ~26.)
            const uint32_t C1 = ~Hx | Sx, C2 = ~Hx & Sx;   // element writes its first / second byte
            const uint32_t *const RK = RKp[c];             // ranks, 4 bytes per dword (element order)
            uint32_t pend = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t X = __builtin_amdgcn_alignbyte(W.w[q + 1], W.w[q], 1u);   // elements 4q..4q+3
                const uint32_t PV = W.w[q];                                                 // the bytes before them
                const uint32_t RQ = __builtin_amdgcn_alignbyte(RK[q], q ? RK[q - 1] : rp0 << 24, 3u);
                const uint32_t PR = 0x88888888u | ((RQ & 0x07070707u) << 4) | (RK[q] & 0x07070707u);
                // bits 4q..4q+3 of a mask -> 0xFF per byte
                auto bytes = [](uint32_t m4) {
                    const uint32_t u = (m4 * 0x204081u) & 0x01010101u;
                    return (u << 8) - u;
                };
                const uint32_t HM = bytes((Hx >> (4 * q)) & 15u), SM = bytes((Sx >> (4 * q)) & 15u);
                const uint32_t B1 = (X & ~SM) | (SM & ((PR & HM) | (PV & ~HM)));
                const uint32_t c1 = (C1 >> (4 * q)) & 15u, c2 = (C2 >> (4 * q)) & 15u;
                const uint2 sl = s_esel[c1 | (c2 << 4)];
                const uint32_t lo = __builtin_amdgcn_perm(X, B1, sl.x), hi = __builtin_amdgcn_perm(X, B1, sl.y);
                const uint32_t L = 8u * (uint32_t)(__popc(c1) + __popc(c2));   // bits out (0..64)
                const uint64_t l64 = (uint64_t)lo << nb, h64 = (uint64_t)hi << nb;
                atomicOr(&s_out32[di], pend | (uint32_t)l64);
                const uint32_t d1 = (uint32_t)(l64 >> 32) | (uint32_t)h64, d2 = (uint32_t)(h64 >> 32);
                const uint32_t nt = nb + L;   // 0..88
                if (nt > 32u) atomicOr(&s_out32[di + 1], d1);
                if (nt > 64u) atomicOr(&s_out32[di + 2], d2);
                pend = nt >= 64u ? d2 : nt >= 32u ? d1 : (pend | (uint32_t)l64);
                di += nt >> 5;
                nb = nt & 31u;
            }
            nb = 0;   // (every bit is in the stage)
        } else {   // M_NYB_DEC / M_NYB_DBODY: compressed byte x, state s = "at the low nybble"
            // Per element (k < kend): its first byte s ? lo : (two ? hi : x), and with two = !s
            // and a hit in the high nybble, a second byte lo; lo = the low nybble's dictionary
            // byte (a hit) or (l & 7) << 4 | the next byte's high nybble, hi = the high nybble's
            // dictionary byte. Four elements at a time in SWAR, the two dictionary lookups as
            // v_perm into the 8-byte table, the output placed as in the encoder above (r4's
            // per-element byte stores: ~26 VALU and 2 LDS byte stores per element).
            const uint32_t T0 = (uint32_t)tblv, T1 = (uint32_t)(tblv >> 32);
            const uint64_t kk0 = M == M_NYB_DBODY ? j0 : j0 + 2;   // stream index of element 0
            const int64_t nvc = (int64_t)len - (int64_t)kk0 - 1;   // elements whose next byte exists
            const uint32_t NV = nvc >= 16 ? 0xFFFFu : nvc <= 0 ? 0u : (1u << (uint32_t)nvc) - 1u;
            const uint32_t IN = kend >= 16 ? 0xFFFFu : (1u << kend) - 1u;
            const uint32_t TW = IN & ~S & fa[c];   // elements writing two bytes (fa: bit 7 of the byte)
            auto bytes = [](uint32_t m4) {       // 4 mask bits -> 0xFF per byte
                const uint32_t u = (m4 * 0x204081u) & 0x01010101u;
                return (u << 8) - u;
            };
            uint32_t pend = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t X = __builtin_amdgcn_alignbyte(W.w[q + 1], W.w[q], 1u);    // elements 4q..4q+3
                const uint32_t NB = __builtin_amdgcn_alignbyte(W.w[q + 1], W.w[q], 2u);   // the bytes after them
                const uint32_t NX = (NB >> 4) & 0x0F0F0F0Fu & bytes((NV >> (4 * q)) & 15u);
                const uint32_t Lb = X & 0x07070707u;
                const uint32_t TL = __builtin_amdgcn_perm(T1, T0, Lb);                     // tbl[l & 7]
                const uint32_t TH = __builtin_amdgcn_perm(T1, T0, (X >> 4) & 0x07070707u);  // tbl[h & 7]
                const uint32_t u3 = (X >> 3) & 0x01010101u, LM = (u3 << 8) - u3;           // low nybble a hit
                const uint32_t LO = (TL & LM) | (((Lb << 4) | NX) & ~LM);
                const uint32_t SM = bytes((S >> (4 * q)) & 15u);
                const uint32_t t4 = (TW >> (4 * q)) & 15u, TM = bytes(t4);
                const uint32_t F = (SM & LO) | (~SM & ((TM & TH) | (~TM & X)));
                const uint32_t c1 = (IN >> (4 * q)) & 15u;
                const uint2 sl = s_esel[c1 | (t4 << 4)];
                const uint32_t lo = __builtin_amdgcn_perm(LO, F, sl.x), hi = __builtin_amdgcn_perm(LO, F, sl.y);
                const uint32_t L = 8u * (uint32_t)(__popc(c1) + __popc(t4));
                const uint64_t l64 = (uint64_t)lo << nb, h64 = (uint64_t)hi << nb;
                atomicOr(&s_out32[di], pend | (uint32_t)l64);
                const uint32_t d1 = (uint32_t)(l64 >> 32) | (uint32_t)h64, d2 = (uint32_t)(h64 >> 32);
                const uint32_t nt = nb + L;
                if (nt > 32u) atomicOr(&s_out32[di + 1], d1);
                if (nt > 64u) atomicOr(&s_out32[di + 2], d2);
                pend = nt >= 64u ? d2 : nt >= 32u ? d1 : (pend | (uint32_t)l64);
                di += nt >> 5;
                nb = nt & 31u;
            }
            nb = 0;
        }
        if (nb) atomicOr(&s_out32[di], (uint32_t)acc);
    }
    __syncthreads();
    // store [o_tile, end): whole granules as uint4, the first and last granule bytewise
    const int64_t end = (int64_t)s_end, beg = (int64_t)o_tile;
    if (end > beg) {
        const int64_t ng = (end - o_al + 15) / 16;
        for (int64_t g = t; g < ng; g += 256) {
            const int64_t b0 = o_al + 16 * g;
            if (b0 >= beg && b0 + 16 <= end) {
                st_nt(reinterpret_cast<uint4 *>(out + b0), *reinterpret_cast<const uint4 *>(s_out + 16 * g));
            } else {
                for (int q = 0; q < 16; ++q) {
                    const int64_t bq = b0 + q;
                    if (bq >= beg && bq < end) out[bq] = s_out[16 * g + q];
                }
            }
        }
    }
}

// Static nybble encode writer, one wave per 4096-element tile (k_nyb_tiles' geometry): lane l
// owns the 64 contiguous elements [64 l, 64 l + 64) of its wave's tile, read as four aligned
// 16-B granules plus the next lane's first dword (DPP; lane 63 loads it), so no per-16-element
// window shuffles; its composition is folded from four 16-element ones (their states from both
// entry states kept for the writer) and scanned across the wave once: no workgroup barrier and
// no cross-wave combination per tile. The four waves of a workgroup share the lookup tables
// only; each stages its tile's output in an LDS row of its own, written as k_fsm_write's SWAR
// writer does (dwords OR-ed at the run's bit offset), then stored as whole granules. ADA: the
// adaptive encode's ranks (aux.rk, element-indexed, 16-B aligned at every 64-element run) with
// the first touches of each 16-element step (step 4 l + b = the lane's block b) settled from its
// k_mtf_resolve record; otherwise the static dictionary. A 16-B aligned input: fsm_run takes
// k_fsm_write otherwise.
template <bool ADA>
__global__ __launch_bounds__(256) void k_nyb_enc_wtile(const uint8_t *__restrict__ in, uint64_t len, uint64_t nelem,
                                                       uint64_t ntiles, const uint64_t *__restrict__ entry,
                                                       const uint4 *__restrict__ loc, const uint64_t *__restrict__ meta,
                                                       uint8_t *__restrict__ out, FsmAux aux)
{
    __shared__ __attribute__((aligned(16))) uint8_t s_out[4][2 * FSM_TILE + 32];
    __shared__ __attribute__((aligned(4))) uint8_t s_rank[256];
    __shared__ uint2 s_esel[256];
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    if (!ADA) fsm_rank_table(s_rank);
    s_esel[t] = make_uint2(c_nyb.esel_lo[t], c_nyb.esel_hi[t]);   // (NybTables)
    const uint64_t T = (uint64_t)blockIdx.x * 4 + (uint64_t)wid;
    const bool live = T < ntiles;
    const uint64_t j0 = T * FSM_TILE + 64 * (uint64_t)lane;   // the lane's first element (stream byte j0 + 1)
    // every global read first: bytes [j0, j0 + 64), the byte after them, (ADA) the ranks, the
    // record count and the first 32 step records (a text tile holds ~24: the records need not
    // wait for the count), the tile's entry
    uint32_t RK[16];   // ranks, 4 per dword (element order)
    uint4 rq0 = make_uint4(0u, 0u, 0u, 0u), rq1 = rq0;
    uint32_t nrec = 0, rk_prev = 0;
    if (ADA) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint64_t k = j0 + 16 * (uint64_t)i;
            const uint4 v = (live && k + 16 <= nelem) ? *reinterpret_cast<const uint4 *>(aux.rk + k)
                                                      : make_uint4(~0u, ~0u, ~0u, ~0u);
            RK[4 * i] = v.x; RK[4 * i + 1] = v.y; RK[4 * i + 2] = v.z; RK[4 * i + 3] = v.w;
        }
        if (aux.frec && live) {
            nrec = aux.fhead[T].x;
            if (lane < 32) {
                const uint4 *const rp = aux.frec + 2 * (T * 128 + (uint64_t)lane);
                rq0 = rp[0];
                rq1 = rp[1];
            }
        }
        if (lane == 0 && live && j0) rk_prev = aux.rk[j0 - 1];   // the tile before's last element, settled in rk
    }
    uint32_t D[17];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t o = j0 + 16 * (uint64_t)i;
        // (plain loads: a wave's four loads each take 16 B of every lane's 64, so a line is read
        // by four instructions; nt loads fetched the tile 1.23x)
        const uint4 g = (live && o < len) ? *reinterpret_cast<const uint4 *>(in + o) : make_uint4(0u, 0u, 0u, 0u);
        D[4 * i] = g.x; D[4 * i + 1] = g.y; D[4 * i + 2] = g.z; D[4 * i + 3] = g.w;
    }
    D[16] = dpp_wave_shl1(D[0]);
    if (lane == 63) D[16] = (live && j0 + 64 < len) ? *reinterpret_cast<const uint32_t *>(in + j0 + 64) : 0u;
    const uint64_t Tc = live ? T : ntiles - 1;
    const uint64_t e = entry[Tc / FSM_GROUP];
    const uint4 lc = loc[Tc];
    const bool whole = aux.whole != 0;
    const uint64_t body = meta[0] + (aux.is_last ? meta[1] : 0);
    if (whole && 2 + body >= len) {   // LITERAL (:1018-1037): ' ' + the raw bytes, one grid-stride pass
        for (uint64_t i = (uint64_t)blockIdx.x * 256 + t; i < len; i += (uint64_t)gridDim.x * 256) out[1 + i] = in[i];
        if (blockIdx.x == 0 && t == 0) out[0] = ' ';
        return;
    }
    if (blockIdx.x == 0 && t == 0 && whole) { out[0] = 0xAF; out[1] = in[0]; }
    __syncthreads();   // s_rank, s_esel
    if (!live) return;   // (whole waves: no barrier below)
    // ranks, and the 16-element blocks' hit masks and states
    uint32_t A[4], V[4], S0[4], S1[4];
    uint32_t comp = FSMP_ID;
    if (!ADA) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const uint32_t X = __builtin_amdgcn_alignbyte(D[q + 1], D[q], 1u);
            RK[q] = (uint32_t)s_rank[X & 255u] | ((uint32_t)s_rank[(X >> 8) & 255u] << 8) |
                    ((uint32_t)s_rank[(X >> 16) & 255u] << 16) | ((uint32_t)s_rank[X >> 24] << 24);
        }
    } else {
        if (j0 < nelem && j0 + 64 > nelem) {   // the stream's last run: its ranks bytewise
            for (uint32_t k = (uint32_t)((nelem - j0) & ~15ull); j0 + k < nelem; ++k) {
                const uint32_t r = aux.rk[j0 + k], sh = 8 * (k & 3), msk = ~(255u << sh);
#pragma unroll
                for (uint32_t q = 0; q < 16; ++q)
                    if ((k >> 2) == q) RK[q] = (RK[q] & msk) | (r << sh);
            }
        }
        if (aux.frec) {   // first touches (0xFE): the settled ranks of the step's record
            // (in the wave's output row, before the row is zeroed: step -> record + 1 at 2 KiB,
            // the records' settled ranks below it)
            uint4 *const s_P = reinterpret_cast<uint4 *>(s_out[wid]);
            uint8_t *const s_map = s_out[wid] + 2048;
            reinterpret_cast<uint32_t *>(s_map)[lane] = 0u;
            __builtin_amdgcn_wave_barrier();
            if (lane < 32 && (uint32_t)lane < nrec) {
                s_map[rq0.z & 255u] = (uint8_t)(lane + 1);
                s_P[lane] = rq1;
            }
            if (__builtin_amdgcn_readfirstlane((int)nrec) > 32) {   // (rare: records past the first 32)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint32_t r = 32u + (uint32_t)lane + 64u * h;
                    if (r < nrec && r < 128u) {   // (MTF_REC)
                        const uint4 *const rp = aux.frec + 2 * (T * 128 + r);
                        const uint4 a = rp[0], b = rp[1];
                        s_map[a.z & 255u] = (uint8_t)(r + 1);
                        s_P[r] = b;
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint32_t mr = s_map[4 * lane + b];
                if (mr) {
                    const uint4 Pv = s_P[mr - 1];
                    const uint32_t p4[4] = {Pv.x, Pv.y, Pv.z, Pv.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint32_t z = RK[4 * b + q] ^ 0xFEFEFEFEu;   // zero bytes: 0xFE ranks
                        const uint32_t m = ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z | 0x7F7F7F7Fu);
                        const uint32_t M = (m >> 7) * 0xFFu;
                        RK[4 * b + q] = (RK[4 * b + q] & ~M) | (p4[q] & M);
                    }
                }
            }
        }
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint64_t kb = j0 + 16 * (uint64_t)b;
        V[b] = kb >= nelem ? 0u : nelem - kb >= 16 ? 0xFFFFu : (1u << (uint32_t)(nelem - kb)) - 1u;
        uint32_t h = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {   // a hit: rank byte < 0x80; 4 byte flags -> 4 bits
            const uint32_t m = (~RK[4 * b + q] >> 7) & 0x01010101u;
            h |= (((m * 0x204081u) >> 21) & 15u) << (4 * q);
        }
        A[b] = h & V[b];
        S0[b] = nyb_enc_states(A[b], V[b], 0u);
        S1[b] = nyb_enc_states(A[b], V[b], 1u);
        const uint32_t miss = ~A[b] & V[b];
        Fsm f;
        f.c0 = __popc(A[b] & S0[b] & 0xFFFFu) + __popc(miss) + __popc(miss & S0[b]);
        f.c1 = __popc(A[b] & S1[b] & 0xFFFFu) + __popc(miss) + __popc(miss & S1[b]);
        f.s0 = (S0[b] >> 16) & 1u;
        f.s1 = (S1[b] >> 16) & 1u;
        comp = fsmp_then(comp, fsmp(f));
    }
    uint32_t xp;
    const uint32_t inc = fsmp_wave_scan(comp, &xp);
    const uint32_t s_g = (uint32_t)(e & 1);
    const uint64_t o_tile = (e >> 1) + (s_g ? lc.y : lc.x) + (whole ? 2 : 0);   // the tile's first output byte
    const uint32_t s_tile = s_g ? lc.w : lc.z;
    const Fsm x = fsmp_unpack(xp), tot = fsmp_unpack((uint32_t)__builtin_amdgcn_readlane((int)inc, 63));
    const uint64_t o0 = o_tile + (s_tile ? x.c1 : x.c0);
    uint32_t st = s_tile ? x.s1 : x.s0;
    const uint64_t s_end = o_tile + (s_tile ? tot.c1 : tot.c0);
    const int64_t o_al = (int64_t)((((uintptr_t)(out + o_tile)) & ~(uintptr_t)15) - (uintptr_t)out);
    uint4 *const so = reinterpret_cast<uint4 *>(s_out[wid]);
    __builtin_amdgcn_wave_barrier();   // (ADA: the records in the row are read)
    for (int i = lane; i < (2 * FSM_TILE + 32) / 16; i += 64) so[i] = make_uint4(0u, 0u, 0u, 0u);
    __builtin_amdgcn_wave_barrier();
    uint32_t *const s_out32 = reinterpret_cast<uint32_t *>(s_out[wid]);
    const uint32_t P = (uint32_t)((int64_t)o0 - o_al);   // stage byte of the lane's first output
    uint32_t di = P >> 2, nb = 8u * (P & 3u), pend = 0;
    // the rank of a hit pending before element 0: the byte before it (ADA: the lane before's last
    // rank; lane 0: the tile before's last element), or the shard's carried one
    uint32_t rp0;
    if (ADA) {
        rp0 = dpp_wave_shr1(RK[15]) >> 24;
        if (lane == 0) rp0 = j0 ? rk_prev : aux.pend_rank;
    } else {
        rp0 = j0 ? (uint32_t)s_rank[D[0] & 255u] : aux.pend_rank;
    }
    uint64_t ob = o0;   // the output byte of the block's first element
    auto bytes = [](uint32_t m4) {   // 4 mask bits -> 0xFF per byte
        const uint32_t u = (m4 * 0x204081u) & 0x01010101u;
        return (u << 8) - u;
    };
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint32_t S = st ? S1[b] : S0[b];
        const uint32_t Hx = A[b] | (~V[b] & 0xFFFFu), Sx = S & V[b];   // (past the input: a hit in state 0)
        const uint32_t C1 = ~Hx | Sx, C2 = ~Hx & Sx;   // element writes its first / second byte
        if (aux.is_last && len >= 2 && len - 2 >= j0 + 16 * (uint64_t)b && len - 2 < j0 + 16 * (uint64_t)b + 16) {
            // odd tail (:1000-1009): the stream's last element a hit left pending: its byte, raw,
            // after the bytes of the elements before it
            const uint32_t kt = (uint32_t)(len - 2 - j0 - 16 * (uint64_t)b);
            if (((Hx & ~Sx) >> kt) & 1u) {
                const uint32_t below = (1u << kt) - 1u;
                const uint32_t k = 16u * (uint32_t)b + kt + 1u;   // its window byte
                uint32_t w = D[0];
#pragma unroll
                for (uint32_t q = 1; q < 17; ++q) w = (k >> 2) == q ? D[q] : w;
                out[ob + __popc(~Hx & below) + __popc(Sx & below)] = (uint8_t)(w >> (8 * (k & 3)));
            }
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
            const int q = 4 * b + qq;
            const uint32_t X = __builtin_amdgcn_alignbyte(D[q + 1], D[q], 1u);   // elements 4q..4q+3
            const uint32_t PV = D[q];                                            // the bytes before them
            const uint32_t RQ = __builtin_amdgcn_alignbyte(RK[q], q ? RK[q - 1] : rp0 << 24, 3u);
            const uint32_t PR = 0x88888888u | ((RQ & 0x07070707u) << 4) | (RK[q] & 0x07070707u);
            const uint32_t HM = bytes((Hx >> (4 * qq)) & 15u), SM = bytes((Sx >> (4 * qq)) & 15u);
            const uint32_t B1 = (X & ~SM) | (SM & ((PR & HM) | (PV & ~HM)));
            const uint32_t c1 = (C1 >> (4 * qq)) & 15u, c2 = (C2 >> (4 * qq)) & 15u;
            const uint2 sl = s_esel[c1 | (c2 << 4)];
            const uint32_t lo = __builtin_amdgcn_perm(X, B1, sl.x), hi = __builtin_amdgcn_perm(X, B1, sl.y);
            const uint32_t nbytes = (uint32_t)(__popc(c1) + __popc(c2));
            const uint64_t l64 = (uint64_t)lo << nb, h64 = (uint64_t)hi << nb;
            atomicOr(&s_out32[di], pend | (uint32_t)l64);
            const uint32_t d1 = (uint32_t)(l64 >> 32) | (uint32_t)h64, d2 = (uint32_t)(h64 >> 32);
            const uint32_t nt = nb + 8u * nbytes;   // 0..88
            if (nt > 32u) atomicOr(&s_out32[di + 1], d1);
            if (nt > 64u) atomicOr(&s_out32[di + 2], d2);
            pend = nt >= 64u ? d2 : nt >= 32u ? d1 : (pend | (uint32_t)l64);
            di += nt >> 5;
            nb = nt & 31u;
            ob += nbytes;
        }
        st = (S >> 16) & 1u;
    }
    __builtin_amdgcn_wave_barrier();
    // store [o_tile, s_end): whole granules as uint4, the first and last granule bytewise
    const int64_t end = (int64_t)s_end, beg = (int64_t)o_tile;
    if (end > beg) {
        const int64_t ng = (end - o_al + 15) / 16;
        const uint8_t *const sb = s_out[wid];
        for (int64_t g = lane; g < ng; g += 64) {
            const int64_t b0 = o_al + 16 * g;
            if (b0 >= beg && b0 + 16 <= end) {
                st_nt(reinterpret_cast<uint4 *>(out + b0), so[g]);
            } else {
                for (int q = 0; q < 16; ++q) {
                    const int64_t bq = b0 + q;
                    if (bq >= beg && bq < end) out[bq] = sb[16 * g + q];
                }
            }
        }
    }
}

// The static nybble decode writer (and the adaptive decode's token pass, aux.tokens) in
// k_nyb_enc_wtile's geometry: a wave per 4096-element tile, 64 contiguous elements (compressed
// bytes j + 2) a lane, the lane's composition folded from four 16-element ones and scanned once;
// the per-element writer is k_fsm_write's decode SWAR form. 16-B aligned input only.
__global__ __launch_bounds__(256) void k_nyb_dec_wtile(const uint8_t *__restrict__ in, uint64_t len, uint64_t nelem,
                                                       uint64_t ntiles, const uint64_t *__restrict__ entry,
                                                       const uint4 *__restrict__ loc, uint8_t *__restrict__ out,
                                                       FsmAux aux)
{
    __shared__ __attribute__((aligned(16))) uint8_t s_out[4][2 * FSM_TILE + 32];
    __shared__ uint2 s_esel[256];
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    s_esel[t] = make_uint2(c_nyb.esel_lo[t], c_nyb.esel_hi[t]);   // (NybTables)
    const uint64_t T = (uint64_t)blockIdx.x * 4 + (uint64_t)wid;
    const bool live = T < ntiles;
    const uint64_t j0 = T * FSM_TILE + 64 * (uint64_t)lane;   // the lane's first element (stream byte j0 + 2)
    uint32_t R[17];   // stream bytes [j0, j0 + 68)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t o = j0 + 16 * (uint64_t)i;
        const uint4 g = (live && o < len) ? *reinterpret_cast<const uint4 *>(in + o) : make_uint4(0u, 0u, 0u, 0u);   // (as above)
        R[4 * i] = g.x; R[4 * i + 1] = g.y; R[4 * i + 2] = g.z; R[4 * i + 3] = g.w;
    }
    R[16] = dpp_wave_shl1(R[0]);
    if (lane == 63) R[16] = (live && j0 + 64 < len) ? *reinterpret_cast<const uint32_t *>(in + j0 + 64) : 0u;
    const uint64_t Tc = live ? T : ntiles - 1;
    const uint64_t e = entry[Tc / FSM_GROUP];
    const uint4 lc = loc[Tc];
    if (blockIdx.x == 0 && t == 0) out[0] = in[1];
    __syncthreads();   // s_esel
    if (!live) return;   // (whole waves: no barrier below)
    uint32_t A[4], B[4], V[4], S0[4], S1[4];
    uint32_t comp = FSMP_ID;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint64_t kb = j0 + 16 * (uint64_t)b;
        V[b] = kb >= nelem ? 0u : nelem - kb >= 16 ? 0xFFFFu : (1u << (uint32_t)(nelem - kb)) - 1u;
        uint32_t h = 0, l = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t X = __builtin_amdgcn_alignbyte(R[4 * b + q + 1], R[4 * b + q], 2u);   // elements 4q..4q+3
            h |= byte_bits4(X, 7) << (4 * q);
            l |= byte_bits4(X, 3) << (4 * q);
        }
        A[b] = h; B[b] = l;
        S0[b] = nyb_dec_states(h, l, V[b], 0u);
        S1[b] = nyb_dec_states(h, l, V[b], 1u);
        Fsm f;
        f.c0 = __popc(V[b]) + __popc(V[b] & h & ~S0[b]);
        f.c1 = __popc(V[b]) + __popc(V[b] & h & ~S1[b]);
        f.s0 = (S0[b] >> 16) & 1u;
        f.s1 = (S1[b] >> 16) & 1u;
        comp = fsmp_then(comp, fsmp(f));
    }
    uint32_t xp;
    const uint32_t inc = fsmp_wave_scan(comp, &xp);
    const uint32_t s_g = (uint32_t)(e & 1);
    const uint64_t o_tile = (e >> 1) + (s_g ? lc.y : lc.x) + 1;   // the tile's first output byte (after out[0])
    const uint32_t s_tile = s_g ? lc.w : lc.z;
    const Fsm x = fsmp_unpack(xp), tot = fsmp_unpack((uint32_t)__builtin_amdgcn_readlane((int)inc, 63));
    const uint64_t o0 = o_tile + (s_tile ? x.c1 : x.c0);
    uint32_t st = s_tile ? x.s1 : x.s0;
    const uint64_t s_end = o_tile + (s_tile ? tot.c1 : tot.c0);
    const int64_t o_al = (int64_t)((((uintptr_t)(out + o_tile)) & ~(uintptr_t)15) - (uintptr_t)out);
    uint4 *const so = reinterpret_cast<uint4 *>(s_out[wid]);
    for (int i = lane; i < (2 * FSM_TILE + 32) / 16; i += 64) so[i] = make_uint4(0u, 0u, 0u, 0u);
    __builtin_amdgcn_wave_barrier();
    uint32_t *const s_out32 = reinterpret_cast<uint32_t *>(s_out[wid]);
    const uint32_t P = (uint32_t)((int64_t)o0 - o_al);
    uint32_t di = P >> 2, nb = 8u * (P & 3u), pend = 0;
    const uint64_t tblv = aux.tokens ? 0x8786858483828180ull : NYB_DICT;   // hit bytes (k_fsm_write)
    const uint32_t T0 = (uint32_t)tblv, T1 = (uint32_t)(tblv >> 32);
    auto bytes = [](uint32_t m4) {   // 4 mask bits -> 0xFF per byte
        const uint32_t u = (m4 * 0x204081u) & 0x01010101u;
        return (u << 8) - u;
    };
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint32_t S = st ? S1[b] : S0[b];
        const int64_t nvc = (int64_t)len - (int64_t)(j0 + 16 * (uint64_t)b + 2) - 1;   // elements whose next byte exists
        const uint32_t NV = nvc >= 16 ? 0xFFFFu : nvc <= 0 ? 0u : (1u << (uint32_t)nvc) - 1u;
        const uint32_t IN = V[b];
        const uint32_t TW = IN & ~S & A[b];   // elements writing two bytes
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
            const int q = 4 * b + qq;
            const uint32_t X = __builtin_amdgcn_alignbyte(R[q + 1], R[q], 2u);    // elements 4q..4q+3
            const uint32_t NB = __builtin_amdgcn_alignbyte(R[q + 1], R[q], 3u);   // the bytes after them
            const uint32_t NX = (NB >> 4) & 0x0F0F0F0Fu & bytes((NV >> (4 * qq)) & 15u);
            const uint32_t Lb = X & 0x07070707u;
            const uint32_t TL = __builtin_amdgcn_perm(T1, T0, Lb);                     // tbl[l & 7]
            const uint32_t TH = __builtin_amdgcn_perm(T1, T0, (X >> 4) & 0x07070707u);  // tbl[h & 7]
            const uint32_t u3 = (X >> 3) & 0x01010101u, LM = (u3 << 8) - u3;           // low nybble a hit
            const uint32_t LO = (TL & LM) | (((Lb << 4) | NX) & ~LM);
            const uint32_t SM = bytes((S >> (4 * qq)) & 15u);
            const uint32_t t4 = (TW >> (4 * qq)) & 15u, TM = bytes(t4);
            const uint32_t F = (SM & LO) | (~SM & ((TM & TH) | (~TM & X)));
            const uint32_t c1 = (IN >> (4 * qq)) & 15u;
            const uint2 sl = s_esel[c1 | (t4 << 4)];
            const uint32_t lo = __builtin_amdgcn_perm(LO, F, sl.x), hi = __builtin_amdgcn_perm(LO, F, sl.y);
            const uint32_t L = 8u * (uint32_t)(__popc(c1) + __popc(t4));
            const uint64_t l64 = (uint64_t)lo << nb, h64 = (uint64_t)hi << nb;
            atomicOr(&s_out32[di], pend | (uint32_t)l64);
            const uint32_t d1 = (uint32_t)(l64 >> 32) | (uint32_t)h64, d2 = (uint32_t)(h64 >> 32);
            const uint32_t nt = nb + L;
            if (nt > 32u) atomicOr(&s_out32[di + 1], d1);
            if (nt > 64u) atomicOr(&s_out32[di + 2], d2);
            pend = nt >= 64u ? d2 : nt >= 32u ? d1 : (pend | (uint32_t)l64);
            di += nt >> 5;
            nb = nt & 31u;
        }
        st = (S >> 16) & 1u;
    }
    __builtin_amdgcn_wave_barrier();
    const int64_t end = (int64_t)s_end, beg = (int64_t)o_tile;
    if (end > beg) {
        const int64_t ng = (end - o_al + 15) / 16;
        const uint8_t *const sb = s_out[wid];
        for (int64_t g = lane; g < ng; g += 64) {
            const int64_t b0 = o_al + 16 * g;
            if (b0 >= beg && b0 + 16 <= end) {
                st_nt(reinterpret_cast<uint4 *>(out + b0), so[g]);
            } else {
                for (int q = 0; q < 16; ++q) {
                    const int64_t bq = b0 + q;
                    if (bq >= beg && bq < end) out[bq] = sb[16 * g + q];
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// Small front-end (small_compression.c:507-665) and its inverse, stateless: each element's
// output (0 or 1 byte encoding, 1 or 2 decoding) depends only on its byte and the bytes
// beside it, so a tile needs only output counts, not the transducer compositions above.
// Geometry: tiles of SM_TILE bytes (per mode, SmMode::tile) on the 16-B address grid of the element bytes (element j
// = byte j + FsmOff of `in`); step s of a tile = 1024 bytes, wave w = its 256-byte quarter,
// lane = one dword (4 elements). A wave's elements are contiguous, so a lane's neighbour
// bytes come from the lanes beside it (ds_bpermute) and only lanes 0 and 63 read a byte of
// the next wave's dwords; all SM_STEPS dword loads of a lane are issued before any is used.
// The writer (k_small_write) uses its own lane-contiguous geometry over the same tiles.
// ------------------------------------------------------------------------------------
template <int M> struct SmMode {
    static constexpr bool dec = (M == M_SMALL_DEC || M == M_SMALL_DBODY);
    static constexpr bool fast = (M == M_SMALL_ENC || M == M_SMALL_BODY0 || M == M_SMALL_BODY1 || dec);
    // tile bytes: 16 KiB for the encoders (the count kernel: 0.238 -> 0.200 ms per GiB of C5
    // text against 8 KiB; the writer equal), 8 KiB for decode (its writer stages up to 2 bytes
    // per element: 33 KiB of LDS at 16 KiB, 4 workgroups per CU, 0.554 against 0.53 ms)
    static constexpr uint32_t tile = dec ? 8192u : 16384u;
    static constexpr int steps = (int)(tile / 1024);
    // the writer's threads: 64 bytes per lane encoding, 32 decoding (measured against 32 / 64:
    // encode 0.53 vs 0.59 ms, decode 0.45 vs 0.45)
    static constexpr int wthreads = (int)(dec ? tile / 32 : tile / 64);
};
#define SM_TILE (SmMode<M>::tile)   /* inside template <int M> code only */
#define SM_STEPS (SmMode<M>::steps)

// tile-relative bounds (uniform, 32-bit): tile byte u = A0 + tile * SM_TILE + u, u in [0, SM_TILE)
struct SmTile {
    int64_t base;          // tile byte 0 relative to `in` (may be negative in tile 0)
    uint32_t lo, hi;       // element bytes: u in [lo, hi)
    uint32_t two;          // u >= two <=> stream byte index >= 2 (a pair may end there)
    uint32_t nxt;          // u < nxt <=> the byte after u is inside the stream
};
template <int M> static __device__ __forceinline__ uint32_t sm_clamp(int64_t v) { return (uint32_t)(v < 0 ? 0 : v > SM_TILE ? SM_TILE : v); }
template <int M> static __device__ __forceinline__ SmTile sm_tile(const uint8_t *in, int off, uint64_t nelem, uint64_t len, uint64_t tile)
{
    const int64_t lead = (int64_t)(((uintptr_t)in + (uintptr_t)off) & 15u);   // element 0's offset in its granule
    SmTile T;
    T.base = (int64_t)off - lead + (int64_t)(tile * SM_TILE);
    T.lo = sm_clamp<M>((int64_t)off - T.base);
    T.hi = sm_clamp<M>((int64_t)off + (int64_t)nelem - T.base);
    T.two = sm_clamp<M>(2 - T.base);
    T.nxt = sm_clamp<M>((int64_t)len - 1 - T.base);
    return T;
}
template <int M> static uint64_t sm_ntiles(const uint8_t *in, int off, uint64_t nelem)
{
    const uint64_t lead = ((uintptr_t)in + (uintptr_t)off) & 15u;
    return nelem ? (lead + nelem + SM_TILE - 1) / SM_TILE : 0;
}

// bytes k of the dword at tile byte u with u + k >= lim / < lim
static __device__ __forceinline__ uint32_t swar_ge(uint32_t u, uint32_t lim)
{
    const uint32_t a = lim > u ? min(lim - u, 4u) : 0u;   // leading bytes below lim
    return a >= 4u ? 0u : 0x80808080u << (8u * a);
}
static __device__ __forceinline__ uint32_t swar_lt(uint32_t u, uint32_t lim)
{
    const uint32_t b = lim > u ? min(lim - u, 4u) : 0u;   // bytes below lim
    return b == 0u ? 0u : 0x80808080u >> (8u * (4u - b));
}

// The 4 elements of a lane's dword d at tile byte u (p / q = the bytes before / after it):
// encode: *val = the output byte of each position, *keep = the positions that emit one;
// decode: *keep = the valid positions (a byte >= 0x80 emits two). Returns the output count.
template <int M, bool INTERIOR>
static __device__ __forceinline__ uint32_t sm_swar(uint32_t d, uint32_t p, uint32_t q, uint32_t u, const SmTile &T,
                                                   uint32_t &val, uint32_t &keep)
{
    const uint32_t valid = INTERIOR ? 0x80808080u : (swar_ge(u, T.lo) & swar_lt(u, T.hi));
    if (SmMode<M>::dec) {
        keep = valid;
        val = d;
        return (uint32_t)__popc(valid) + (uint32_t)__popc(valid & d & 0x80808080u);
    }
    const uint32_t prev = (d << 8) | p, next = (d >> 8) | (q << 24);
    uint32_t second = swar_eq(prev, 0x20202020u) & swar_lower(d);
    if (!INTERIOR && M != M_SMALL_BODY1) second &= swar_ge(u, T.two);   // stream bytes 0-1 never pair
    uint32_t start = swar_eq(d, 0x20202020u) & swar_lower(next);
    if (!INTERIOR) start &= swar_lt(u, T.nxt);   // the next byte must be inside the stream
    const uint32_t m8 = (start - (start >> 7)) | start;   // 0x80 -> 0xFF per byte
    val = (d & ~m8) | ((next | 0x80808080u) & m8);       // ' ' + letter -> 0x80 + letter
    keep = valid & ~second;
    return (uint32_t)__popc(keep);
}

// the lane's 16 dwords (step st: tile byte st * 1024 + w * 256 + 4 lane), all loads issued
// before any is used; the bytes at the waves' edges go through LDS (SmEdge), with one byte
// before and after the tile read from memory
template <int M>
static __device__ __forceinline__ void sm_load(const uint8_t *__restrict__ in, uint64_t len, const SmTile &T, int w,
                                               int lane, uint32_t (&dv)[SM_STEPS])
{
    const uint32_t ulo = T.lo ? T.lo - 1 : 0, uhi = T.hi + 1;   // bytes the elements read
#pragma unroll
    for (int st = 0; st < SM_STEPS; ++st) {
        const uint32_t u = (uint32_t)(st * 1024 + w * 256 + lane * 4);
        const int64_t o = T.base + (int64_t)u;   // relative to in
        dv[st] = (u + 4 > ulo && u < uhi && o + 4 > 0 && o < (int64_t)len)
                     ? __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(in + o)) : 0u;
    }
}
template <int M> struct SmEdge {
    uint8_t first[SM_STEPS][4], last[SM_STEPS][4];   // each wave's first / last byte per step
    uint8_t before, after;                            // the bytes beside the tile
};
template <int M>
static __device__ __forceinline__ void sm_edges_put(SmEdge<M> &E, const uint8_t *__restrict__ in, uint64_t len,
                                                    const SmTile &T, int t, const uint32_t (&dv)[SM_STEPS])
{
    const int lane = t & 63, w = t >> 6;
    if (lane == 0 || lane == 63) {
#pragma unroll
        for (int st = 0; st < SM_STEPS; ++st) {
            if (lane == 0) E.first[st][w] = (uint8_t)dv[st];
            else E.last[st][w] = (uint8_t)(dv[st] >> 24);
        }
    }
    if (t == 0) E.before = (T.base - 1 >= 0 && T.base - 1 < (int64_t)len) ? in[T.base - 1] : 0;
    if (t == 255) E.after = (T.base + SM_TILE >= 0 && T.base + SM_TILE < (int64_t)len) ? in[T.base + SM_TILE] : 0;
}
// bytes before / after the lane's dword at step st (after a barrier behind sm_edges_put):
// x = before, y = after; branch-free (the wave-edge bytes are uniform broadcast reads)
template <int M>
static __device__ __forceinline__ uint2 sm_nb(const SmEdge<M> &E, uint32_t d, int st, int w, int lane)
{
    // the neighbour lanes' dwords by DPP wave shifts (VALU; the bpermutes they replace were a
    // fifth of the writer's LDS instructions)
    const uint32_t pu = dpp_wave_shr1(d) >> 24, qd = dpp_wave_shl1(d) & 255u;
    const uint32_t pe = w > 0 ? E.last[st][w - 1] : st > 0 ? E.last[st - 1][3] : E.before;
    const uint32_t qe = w < 3 ? E.first[st][w + 1] : st + 1 < SM_STEPS ? E.first[st + 1][0] : E.after;
    return make_uint2(lane == 0 ? pe : pu, lane == 63 ? qe : qd);
}

// One tile per workgroup. (A persistent grid with the next tile's loads issued ahead
// measured 1.6-1.8x slower: 150-246 VGPRs, 2-3 waves per SIMD.)
template <int M>
__global__ __launch_bounds__(256) void k_small_tiles(const uint8_t *__restrict__ in, uint64_t len, uint64_t nelem,
                                                     uint4 *__restrict__ summ)
{
    __shared__ uint32_t s_w[4];
    __shared__ SmEdge<M> E;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const SmTile T = sm_tile<M>(in, FsmOff<M>::v, nelem, len, blockIdx.x);
    uint32_t dv[SM_STEPS];
    sm_load<M>(in, len, T, w, lane, dv);
    if (!SmMode<M>::dec) {
        sm_edges_put<M>(E, in, len, T, t, dv);
        __syncthreads();
    }
    uint32_t cnt = 0;
    const bool interior = T.lo == 0 && T.hi == SM_TILE && T.two == 0 && T.nxt == SM_TILE;
#pragma unroll
    for (int st = 0; st < SM_STEPS; ++st) {
        const uint2 nb = SmMode<M>::dec ? make_uint2(0u, 0u) : sm_nb<M>(E, dv[st], st, w, lane);
        const uint32_t u = (uint32_t)(st * 1024 + w * 256 + lane * 4);
        uint32_t val, keep;
        cnt += interior ? sm_swar<M, true>(dv[st], nb.x, nb.y, u, T, val, keep)
                        : sm_swar<M, false>(dv[st], nb.x, nb.y, u, T, val, keep);
    }
    const uint32_t tot = wave_scan_incl(cnt);
    if (lane == 63) s_w[w] = tot;
    __syncthreads();
    if (t == 0) {
        const uint32_t c = s_w[0] + s_w[1] + s_w[2] + s_w[3];
        summ[blockIdx.x] = make_uint4(c, c, 0u, 0u);   // a stateless composition
    }
}

// The C5 decode's tile summaries without a counting pass (dc_small_huff_decode): the decoder
// counted the symbols >= 0x80 of every group of 4096 (gexp; S = 64), and a decode tile (8 KiB of
// the front-end stream, 16-B aligned) is two groups: output bytes = its elements + those
// symbols (the raw first byte M[1] excluded). Thread 0 also hands the type byte M[0] to the
// host (meta[8]: only 8 = EIGHT_BIT_PRUNED is decoded this way).
__global__ __launch_bounds__(256) void k_small_dec_summ(const uint32_t *__restrict__ gexp, uint64_t ngroups,
                                                        const uint8_t *__restrict__ in, uint64_t len, uint64_t ntiles,
                                                        uint4 *__restrict__ summ, uint64_t *__restrict__ meta)
{
    const uint64_t tile = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (tile == 0) meta[8] = in[0];
    if (tile >= ntiles) return;
    constexpr uint64_t TB = SmMode<M_SMALL_DEC>::tile;
    static_assert(TB == 2 * 64 * DC_SYNC_GROUP, "a decode tile is two groups of S = 64");
    const uint64_t lo = tile * TB > 2 ? tile * TB : 2, hi = (tile + 1) * TB < len ? (tile + 1) * TB : len;
    uint32_t c = hi > lo ? (uint32_t)(hi - lo) : 0u;
    c += gexp[2 * tile] + (2 * tile + 1 < ngroups ? gexp[2 * tile + 1] : 0u);
    if (tile == 0 && len > 1 && in[1] >= 0x80) c -= 1;   // M[1] = x[0], raw (small_compression.c:587)
    summ[tile] = make_uint4(c, c, 0u, 0u);
}

// The writer: lane-contiguous geometry (unlike the count kernel's, whose tile totals are the
// same): wave w owns bytes [w * WB, +WB) of the tile and lane l its LB contiguous bytes, so
// a lane's output is one contiguous run. The lane packs its kept bytes into a 64-bit accumulator and ORs whole dwords into the zeroed LDS stage (ds_or_b32: the
// dwords it shares with its neighbours' runs merge without ordering). One dword store per 4
// output bytes instead of one byte store per element (per GiB of C5 text: decode 0.51 -> 0.45
// ms; encode equal, 0.53).
template <int M>
__global__ __launch_bounds__(SmMode<M>::wthreads) void k_small_write(const uint8_t *__restrict__ in, uint64_t len, uint64_t nelem,
                                                     const uint64_t *__restrict__ entry, const uint4 *__restrict__ loc,
                                                     const uint64_t *__restrict__ meta, uint8_t *__restrict__ out)
{
    constexpr bool dec = SmMode<M>::dec;
    constexpr uint32_t NT = SmMode<M>::wthreads, NW = NT / 64;
    constexpr uint32_t TILE = SM_TILE, WB = TILE / NW, LB = TILE / NT, LD = LB / 4;
    constexpr uint32_t SW = ((dec ? 2 * TILE : TILE) + 32) / 4;   // stage dwords: output + lead + flush slack
    static_assert(LB % 16 == 0 && SW % 4 == 0, "uint4 geometry");
    __shared__ uint32_t s_w[NW];
    __shared__ uint8_t s_first[NW], s_last[NW], s_before, s_after;
    __shared__ __attribute__((aligned(16))) uint32_t s_out[SW];
    __shared__ uint2 s_sel[16];   // decode: v_perm selectors of the 4-8 output bytes of a dword, per pair pattern
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const bool enc = M == M_SMALL_ENC;
    if (dec && t < 16) s_sel[t] = make_uint2(c_nyb.dsel_lo[t], c_nyb.dsel_hi[t]);   // (NybTables)
    const uint64_t total = enc ? 2 + meta[0] : 1 + meta[0];
    if (enc && total >= len) {   // LITERAL: ' ' + raw input (:655-662), one grid-stride pass
        for (uint64_t i = (uint64_t)blockIdx.x * NT + t; i < len; i += (uint64_t)gridDim.x * NT) out[1 + i] = in[i];
        if (blockIdx.x == 0 && t == 0) out[0] = ' ';
        return;
    }
    const bool headed = !FsmMode<M>::body;
    if (blockIdx.x == 0 && t == 0 && headed) {
        if (enc) { out[0] = 8; out[1] = in[0]; }
        else out[0] = in[1];
    }
    const SmTile T = sm_tile<M>(in, FsmOff<M>::v, nelem, len, blockIdx.x);
    const uint32_t u0 = (uint32_t)w * WB + (uint32_t)lane * LB;   // the lane's first tile byte
    uint32_t d[LD];
    {
        const uint32_t ulo = T.lo ? T.lo - 1 : 0, uhi = T.hi + 1;   // bytes the elements read
#pragma unroll
        for (uint32_t k = 0; k < LD / 4; ++k) {
            const uint32_t u = u0 + 16 * k;
            const int64_t o = T.base + (int64_t)u;   // relative to in; in + T.base is 16-B aligned
            const uint4 v = (u + 16 > ulo && u < uhi && o + 16 > 0 && o < (int64_t)len)
                                ? ld_nt(reinterpret_cast<const uint4 *>(in + o)) : make_uint4(0u, 0u, 0u, 0u);
            d[4 * k] = v.x; d[4 * k + 1] = v.y; d[4 * k + 2] = v.z; d[4 * k + 3] = v.w;
        }
    }
#pragma unroll
    for (uint32_t k = 0; k < SW / 4 / NT + 1; ++k)   // zero the stage (ordered before the ORs by the barrier below)
        if (t + NT * k < SW / 4) reinterpret_cast<uint4 *>(s_out)[t + NT * k] = make_uint4(0u, 0u, 0u, 0u);
    uint32_t p = 0, q = 0;   // the bytes before / after the lane's run
    if (!dec) {
        if (lane == 0) s_first[w] = (uint8_t)d[0];
        if (lane == 63) s_last[w] = (uint8_t)(d[LD - 1] >> 24);
        if (t == 0) s_before = (T.base - 1 >= 0 && T.base - 1 < (int64_t)len) ? in[T.base - 1] : 0;
        if (t == (int)NT - 1) s_after = (T.base + TILE >= 0 && T.base + TILE < (int64_t)len) ? in[T.base + TILE] : 0;
        __syncthreads();
        const uint32_t pu = dpp_wave_shr1(d[LD - 1]) >> 24, qd = dpp_wave_shl1(d[0]) & 255u;
        p = lane == 0 ? (w > 0 ? s_last[w - 1] : s_before) : pu;
        q = lane == 63 ? (w + 1 < (int)NW ? s_first[w + 1] : s_after) : qd;
    }
    const bool interior = T.lo == 0 && T.hi == TILE && T.two == 0 && T.nxt == TILE;
    auto swar = [&](uint32_t k, uint32_t &val, uint32_t &keep) -> uint32_t {
        const uint32_t pk = k > 0 ? d[k - 1] >> 24 : p, qk = k + 1 < LD ? d[k + 1] & 255u : q;
        const uint32_t u = u0 + 4 * k;
        return interior ? sm_swar<M, true>(d[k], pk, qk, u, T, val, keep) : sm_swar<M, false>(d[k], pk, qk, u, T, val, keep);
    };
    uint32_t cnt = 0, vals[LD], keeps[LD];
#pragma unroll
    for (uint32_t k = 0; k < LD; ++k) cnt += swar(k, vals[k], keeps[k]);
    const uint32_t incl = wave_scan_incl(cnt);
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    uint32_t pre = 0, run = 0;
#pragma unroll
    for (int x = 0; x < (int)NW; ++x) {
        const uint32_t v = s_w[x];
        pre += x < w ? v : 0u;
        run += v;
    }
    const uint64_t e = entry[blockIdx.x / FSM_GROUP];
    const uint64_t o_tile = (e >> 1) + loc[blockIdx.x].x + (headed ? (enc ? 2 : 1) : 0);   // first output byte
    const int64_t o_al = (int64_t)((((uintptr_t)(out + o_tile)) & ~(uintptr_t)15) - (uintptr_t)out);
    const uint32_t lead = (uint32_t)((int64_t)o_tile - o_al);   // stage offset of the tile's first byte
    if (dec && interior) {
        // Decode, a tile with every byte an element (all but the stream's first and last
        // tiles): per input dword, its 4 bytes expand to 4-8 by two v_perm (selectors by the
        // pattern of its bytes >= 0x80, from s_sel), and the lane's run advances by whole
        // dwords: OR-ed into the stage at the run's bit offset, the partial last dword too (ORs
        // are idempotent, so the pending bits are OR-ed again with the next ones: no flush
        // branch). ~20 VALU per input dword where the per-byte loop below takes ~60.
        const uint32_t P = lead + pre + incl - cnt;
        uint32_t di = P >> 2, nb = 8u * (P & 3u), pend = 0;
#pragma unroll
        for (uint32_t k = 0; k < LD; ++k) {
            const uint32_t x = vals[k], h = x & 0x80808080u;
            uint32_t m = h >> 7;                  // bits 0, 8, 16, 24
            m |= m >> 7;                          // + 1, 9, 17
            m = (m | (m >> 14)) & 15u;            // the pattern
            const uint2 sl = s_sel[m];
            const uint32_t lo = __builtin_amdgcn_perm(x ^ h, 0x20202020u, sl.x);
            const uint32_t hi = __builtin_amdgcn_perm(x ^ h, 0x20202020u, sl.y);
            const uint32_t hb = 8u * (uint32_t)__popc(h);   // bits of hi (0..32)
            const uint64_t l64 = (uint64_t)lo << nb, h64 = (uint64_t)hi << nb;
            atomicOr(&s_out[di], pend | (uint32_t)l64);                      // always whole
            const uint32_t d1 = (uint32_t)(l64 >> 32) | (uint32_t)h64;       // nb + hb bits
            atomicOr(&s_out[di + 1], d1);
            const uint32_t nt = nb + hb;                                      // 0..56
            const bool full = nt >= 32u;
            if (nt > 32u) atomicOr(&s_out[di + 2], (uint32_t)(h64 >> 32));   // (rare: many pairs)
            pend = full ? (uint32_t)(h64 >> 32) : d1;
            di += full ? 2u : 1u;
            nb = nt & 31u;
        }
    } else {   // the lane's run: from stage byte P, packed 4 bytes to a dword
        const uint32_t P = lead + pre + incl - cnt;
        uint32_t di = P >> 2, nb = 8u * (P & 3u);
        uint64_t acc = 0;
        auto flush = [&]() {
            if (nb >= 32u) {
                atomicOr(&s_out[di], (uint32_t)acc);
                acc >>= 32;
                nb -= 32u;
                ++di;
            }
        };
#pragma unroll
        for (uint32_t k = 0; k < LD; ++k) {
            const uint32_t val = vals[k], keep = keeps[k];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint32_t on = (keep >> (8 * b + 7)) & 1u, v = (val >> (8 * b)) & 255u;
                if (dec) {   // >= 0x80: ' ' then the letter
                    const uint32_t two = v >> 7;
                    const uint32_t piece = two ? (0x20u | ((v & 0x7Fu) << 8)) : v;
                    acc |= (uint64_t)(on ? piece : 0u) << nb;
                    nb += on ? (two ? 16u : 8u) : 0u;
                    if (b & 1) flush();   // <= 32 bits per 2 elements
                } else {
                    acc |= (uint64_t)(on ? v : 0u) << nb;
                    nb += on ? 8u : 0u;
                }
            }
            if (!dec) flush();   // <= 32 bits per dword
        }
        if (nb) atomicOr(&s_out[di], (uint32_t)acc);
    }
    __syncthreads();
    // store [o_tile, o_tile + run): whole granules as uint4, the first and last bytewise
    const uint8_t *stage = reinterpret_cast<const uint8_t *>(s_out);
    const int64_t beg = (int64_t)o_tile, end = beg + (int64_t)run;
    if (end > beg) {
        const int64_t ng = (end - o_al + 15) / 16;
        for (int64_t g = t; g < ng; g += NT) {
            const int64_t b0 = o_al + 16 * g;
            if (b0 >= beg && b0 + 16 <= end) {
                st_nt(reinterpret_cast<uint4 *>(out + b0), *reinterpret_cast<const uint4 *>(stage + 16 * g));
            } else {
                for (int k = 0; k < 16; ++k) {
                    const int64_t bq = b0 + k;
                    if (bq >= beg && bq < end) out[bq] = stage[16 * g + k];
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// Adaptive nybble encode, in parallel (SURVEY.md N4 [verified P6]). The move-to-front list of
// context c after a stretch of input is the first 8 distinct of (that stretch's context-c
// bytes, newest first) followed by the list before it. So "the list state after a tile,
// started empty" is a summary, and summaries compose associatively:
//     after(A then B)_c = first-8-distinct(B_c ++ A_c)
// = touching B_c's entries, oldest first, on top of A_c. The encoder's rank of byte i is its
// position in the list before the touch (compress_byte_index :833-839, update_context
// :665-687). Pipeline: k_mtf_walk<2> walks each 4096-element tile once from empty lists (one
// lane per tile, the 16 lists as u64 words in LDS): the tile summary, and every rank (0..7,
// 0xFF = miss) that does not depend on the entry lists, the others (first touches) listed;
// k_mtf_reduce composes 64 summaries per group, level by level; k_mtf_down hands each child its
// entry lists from the top (the initial " etaoins" lists, or a shard's entry lists);
// k_mtf_resolve settles the first touches and composes the transducer's tile summaries; the
// ranks drive k_fsm_write<M_NYB_ENC>. (k_mtf_walk<0>: summaries only, for shard plans.)
// ------------------------------------------------------------------------------------
#define MTF_TILE 4096
#define MTF_FAN 64
struct MtfSum {
    uint64_t L[16];    // list of context c: byte k = entry k (most recent first)
    uint8_t cnt[16];   // valid entries per list (0..8)
};

// move v to the front of (L, cnt); returns v's rank before the touch, or -1 (miss)
static __device__ __forceinline__ int mtf_touch64(uint64_t &L, uint32_t &cnt, uint32_t v)
{
    const uint64_t ones = 0x0101010101010101ull;
    const uint64_t t = L ^ (ones * v);
    const uint64_t z = (t - ones) & ~t & (ones << 7);   // lowest flagged byte is the first match
    const int pos = z ? (int)(__builtin_ctzll(z) >> 3) : 8;
    const bool hit = pos < (int)cnt;
    const int p = hit ? pos : (cnt < 7 ? (int)cnt : 7);   // entry dropped: the match, or the last slot
    const uint64_t low = (1ull << (8 * p)) - 1;           // entries above p stay, [0, p) move up
    const uint64_t high = p == 7 ? 0ull : ~((1ull << (8 * (p + 1))) - 1);
    L = (L & high) | ((L & low) << 8) | (uint64_t)v;
    if (!hit && cnt < 8) ++cnt;
    return hit ? pos : -1;
}

// apply a summary list (newest first, n entries) on top of (L, cnt): the same list as touching
// S's entries oldest first, by composition: S's entries, then L's first cnt entries that are not
// among them (each an independent SWAR test), packed, to 8 (r4: 8 dependent touches per child,
// ~30 VALU each, took k_mtf_reduce + k_mtf_down to 0.17 ms per GiB)
static __device__ __forceinline__ void mtf_apply(uint64_t &L, uint32_t &cnt, uint64_t S, uint32_t n)
{
    constexpr uint64_t ones = 0x0101010101010101ull;
    const uint64_t inS = n >= 8 ? ~0ull : (1ull << (8 * n)) - 1ull;   // S's bytes
    const uint64_t Sm = S & inS;
    uint64_t C = 0;
    uint32_t pos = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t a = (uint32_t)(L >> (8 * k)) & 255u;
        const uint64_t t = Sm ^ (ones * a);
        // a zero byte of t among S's bytes (flags above the range are masked: a false flag only
        // sits above a true zero byte)
        const uint64_t z = (t - ones) & ~t & (ones << 7) & inS;
        const bool keep = (uint32_t)k < cnt && z == 0ull;
        C |= keep ? (uint64_t)a << (8 * pos) : 0ull;
        pos += keep ? 1u : 0u;
    }
    L = Sm | (n < 8 ? C << (8 * n) : 0ull);
    cnt = min(8u, n + pos);
}

// move v to the front of a full list (8 entries): mtf_touch64 with cnt = 8. On a list of cnt < 8
// entries padded with zero bytes it leaves the same entries as mtf_touch64 with that cnt (a miss
// drops the last byte, a pad; a zero v finds the first pad, the byte a miss would drop).
// pb = 8 pos + 7 for a match at pos (63 for a miss too); hit = a match.
static __device__ __forceinline__ uint64_t mtf_touch8(uint64_t L, uint32_t v, uint32_t &pb, bool &hit)
{
    const uint32_t vb = __builtin_amdgcn_perm(0u, v, 0u);   // v in every byte (no 32-bit multiply)
    const uint32_t tl = (uint32_t)L ^ vb, th = (uint32_t)(L >> 32) ^ vb;
    const uint64_t d = (((uint64_t)th << 32) | tl) - 0x0101010101010101ull;
    const uint32_t zl = (uint32_t)d & ~tl & 0x80808080u, zh = (uint32_t)(d >> 32) & ~th & 0x80808080u;
    hit = (zl | zh) != 0u;   // the lowest flag is the first match
    pb = (uint32_t)__builtin_ctzll(((uint64_t)(zh | 0x80000000u) << 32) | zl);
    const uint64_t m = ~0ull >> (63u - pb);   // bytes [0, pos]: up by one, v in at 0
    return (((L << 8) | v) & m) | (L & ~m);
}

// mtf_touch8 of byte k of X (k a constant), returning 8 x the match position (56 for a miss) in
// place of pb: the byte is never extracted (it is broadcast, and shifted in under the list, by
// byte permutes); the moved bytes [0, pos] are z ^ (z - 1) of the match flags z (all bytes for a
// miss, z = 0) and pos their popcount / 8 - 1 (12 VALU ops where ctz and a shifted mask took 14)
static __device__ __forceinline__ uint64_t mtf_touch8x(uint64_t L, uint32_t X, uint32_t k, uint32_t &pos8, bool &hit)
{
    const uint32_t vb = __builtin_amdgcn_perm(0u, X, k * 0x01010101u);
    const uint32_t Ll = (uint32_t)L, Lh = (uint32_t)(L >> 32);
    const uint32_t tl = Ll ^ vb, th = Lh ^ vb;
    const uint64_t d = (((uint64_t)th << 32) | tl) - 0x0101010101010101ull;
    const uint32_t zl = (uint32_t)d & ~tl & 0x80808080u, zh = (uint32_t)(d >> 32) & ~th & 0x80808080u;
    const uint64_t z = ((uint64_t)zh << 32) | zl, m = z ^ (z - 1ull);   // the lowest flag is the first match
    hit = z != 0ull;
    // pos8 = 8 pos: popcount(m) - 8 as two accumulating v_bcnt (the compiler adds them with a third op)
    asm("v_bcnt_u32_b32 %0, %1, -8\n\tv_bcnt_u32_b32 %0, %2, %0" : "=&v"(pos8) : "v"((uint32_t)m), "v"((uint32_t)(m >> 32)));
    const uint32_t sl = __builtin_amdgcn_perm(Ll, X, 0x06050400u | k);   // (L << 8 | x), low dword
    const uint32_t sh = __builtin_amdgcn_alignbyte(Lh, Ll, 3u);          // (L << 8), high dword
    return ((((uint64_t)sh << 32) | sl) & m) | (L & ~m);
}

// k_mtf_walk: one pass over each 4096-element tile from EMPTY lists (elements are bytes 1..len-1
// of `in`: element e = byte e+1, its context byte e). MODE 0: the tile summaries -> summ[tile].
// MODE 2: also the ranks into rk, but for the FIRST TOUCHES (MODE + 1: the same for an input of any
// alignment, with the dword selects an unaligned tile start needs). A hit's rank is final already (an
// entry touched in the tile sits above every entry-list byte, in the same order whatever the
// entry lists were); a miss on a full list is a miss (0xFF); a miss while the list holds fewer
// than 8 entries is a first touch, whose rank depends on the entry lists: it is written 0xFE, and
// each 16-element step that holds one is listed for k_mtf_resolve as a STEP RECORD of two uint4:
// (the nybble encoder's composition of the steps since the previous record, hits | first
// touches << 16, step | context byte of its element 0 << 8 | elements << 16, 0), and the step's
// 16 element bytes. head[tile] = (records, the composition after the last one). (The encoder's
// FSM tiles are these tiles; a step is a lane of its writer.)
// A lane walks its tile with the 16 lists in LDS (column t). Per element: the touched list is
// written back, then the next element's list read (its context is this element's byte; the
// same address returns the list just written: no compare and selects); the other 3 waves of a
// SIMD cover the round trip (r5: 26 -> 23 VALU per element, 1.128 -> 1.117 ms per GiB, against
// reading it before the write, profiles/r5walk2_mtf_walk_raw_ab.log); the input
// comes in 16-B granules loaded a 64-element group ahead. 23 VALU per element in all (r4: 35,
// 1.311 ms per GiB, profiles/r5walk_mtf_walk_valu_ab.log). Lists are padded with zero bytes
// (mtf_touch8), so a list is short while its last byte is 0 and its count is 8 - its zero bytes,
// both exact while no element is a zero byte; a tile that has one is walked again with counts
// (mtf_touch64). (r4 before: a summary pass, then a second walk of every tile from its entry
// lists for the ranks, 0.90 + 1.24 ms per GiB; first: one lane-local loop that waited on every
// list read and on the granule just loaded, 1.64 + 2.03 ms.)
#define MTF_REC 128   /* step records per tile: <= its first touches, <= 8 per context */

static_assert(FSM_TILE == MTF_TILE, "k_mtf_walk<2> composes the nybble encoder's tile summaries");
template <int MODE>
__global__ __launch_bounds__(256) void k_mtf_walk(
    const uint8_t *__restrict__ in, uint64_t len, uint64_t ntiles, MtfSum *__restrict__ summ, uint8_t *__restrict__ rk,
    uint4 *__restrict__ rec, uint2 *__restrict__ head)
{
    static_assert(MODE >= 0 && MODE <= 3, "summaries (0), or summaries and ranks (2); + 1: any input alignment");
    constexpr bool RANKS = MODE >= 2, GEN = (MODE & 1) != 0;
    __shared__ uint64_t s_L[16][256];
    const int t = threadIdx.x;
    const uint64_t tile = (uint64_t)blockIdx.x * 256 + t;
    if (tile >= ntiles) return;   // no barriers below
    const uint64_t e0 = tile * MTF_TILE;
    const uint64_t e1 = (e0 + MTF_TILE < len - 1) ? e0 + MTF_TILE : len - 1;   // elements [e0, e1)
    for (int c = 0; c < 16; ++c) s_L[c][t] = 0ull;
    const uint32_t prev0 = in[e0];
    uint32_t cc = (prev0 >> 3) & 15u;
    uint64_t Lc = 0ull;
    uint32_t anyz = 0;   // 0x80 bits: a zero byte among the tile's elements
    uint32_t accp = FSMP_ID, nrec = 0;
    uint4 *const trec = rec + (RANKS ? 2 * tile * MTF_REC : 0);
    // MODE 2, after 16 elements (element k: rank byte k of R, byte k of X, valid bits nv): a step
    // without first touches folds into accp, one with them is listed (two 16-B stores: the
    // per-first-touch list with its segment folds measured 0.38 ms per GiB in divergent branches)
    auto post = [&](const uint32_t (&R)[4], const uint32_t (&X)[4], uint32_t pv, uint64_t e, uint32_t nv) {
        uint32_t H = 0, F = 0;   // hits (a byte <= 7); first touches (0xFE)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            H |= byte_bits4(~R[q], 7) << (4 * q);
            F |= byte_bits4(R[q] & ~(R[q] << 7), 7) << (4 * q);
        }
        F &= nv;
        if (F) {
            // (<= 128 records, but for a walk with a zero byte, whose pads are ambiguous: its list
            // is rebuilt by the counted walk; the bound keeps it off the next tile's)
            if (nrec < MTF_REC) {
                trec[2 * nrec] = make_uint4(accp, H | (F << 16), (uint32_t)((e - e0) >> 4) | (pv << 8) | (__popc(nv) << 16), 0u);
                trec[2 * nrec + 1] = make_uint4(X[0], X[1], X[2], X[3]);
            }
            ++nrec;
            accp = FSMP_ID;
        } else {
            accp = fsmp_then(accp, fsmp(nyb_lane_fsm<M_NYB_ENC>(H, 0u, nv)));
        }
    };
    // granule i = bytes [gb + 16 i, +16) of `in`, gb = element e0's byte rounded down to 16 B;
    // element e0 + 16 s + k is byte sh + 16 s + k of granules s, s + 1 (sh uniform: in + 1's
    // alignment, e0 a multiple of 16)
    const uint64_t a = (uintptr_t)in & 15u, gb = ((e0 + 1 + a) & ~15ull) - a;
    const uint32_t sh = (uint32_t)((e0 + 1 + a) & 15u), dq = sh >> 2, db = sh & 3u;
    auto ld = [&](uint64_t i) {
        const int64_t o = (int64_t)(gb + 16 * i);   // (-a .. : granule 0 may begin before in)
        return o < (int64_t)len ? *reinterpret_cast<const uint4 *>(in + o) : make_uint4(0u, 0u, 0u, 0u);
    };
    auto step = [&](const uint4 &A, const uint4 &B, uint64_t e, uint4 &Rout) {
        const uint32_t d8[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
        uint32_t X[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {   // dwords dq + j, dq + j + 1 (dq uniform: selects, GEN only)
            uint32_t lo = d8[j], hi = d8[j + 1];
            if (GEN) {
#pragma unroll
                for (int k = 1; k < 4; ++k) { lo = dq == (uint32_t)k ? d8[j + k] : lo; hi = dq == (uint32_t)k ? d8[j + k + 1] : hi; }
            }
            X[j] = __builtin_amdgcn_alignbyte(hi, lo, db);
            anyz |= (X[j] - 0x01010101u) & ~X[j] & 0x80808080u;
        }
        const uint32_t pv = (cc << 3);   // (context of element 0: only its bits 3..6 are used)
        uint32_t R[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            uint32_t cn;   // (x >> 3) & 15 of byte x: one v_bfe (the compiler splits a ubfe into a shift and a mask)
            asm("v_bfe_u32 %0, %1, %2, 4" : "=v"(cn) : "v"(X[k >> 2]), "n"(8 * (k & 3) + 3));
            uint32_t p8;   // 8 x the match position
            bool hit;
            const uint64_t L2 = mtf_touch8x(Lc, X[k >> 2], (uint32_t)(k & 3), p8, hit);
            s_L[cc][t] = L2;
            if (RANKS) {   // the rank, 8 x, into byte k & 3 (a shift by 8 (k & 3) - 3 takes out the 8)
                const uint32_t r8 = hit ? p8 : (Lc >> 56) == 0ull ? 0xFEu << 3 : 0xFFu << 3;
                R[k >> 2] |= (k & 3) ? r8 << (8 * (k & 3) - 3) : r8 >> 3;
                asm volatile("" : "+v"(R[k >> 2]));   // (sunk to the step's end, 16 ranks' inputs stayed live: +56 VGPRs)
            }
            Lc = s_L[cn][t];   // the next element's list, after this write (the same context: L2)
            cc = cn;
        }
        if (RANKS) {
            Rout = make_uint4(R[0], R[1], R[2], R[3]);   // (stored by the group: 64 B at once)
            post(R, X, pv, e, 0xFFFFu);
        }
    };
    // 64 elements (granules A..E: their bytes start sh into A): 4 steps, then the 64 ranks as one
    // 64-B burst (16-B pieces of lines, one per step and lane, left the walk at 2.7x its
    // algorithmic write traffic)
    auto quad = [&](const uint4 &A, const uint4 &B, const uint4 &C, const uint4 &D, const uint4 &E, uint64_t ee) {
        // (the steps kept apart: interleaved by the scheduler they held 155 VGPRs, 3 waves per SIMD)
        uint4 Ra, Rb, Rc, Rd;
        step(A, B, ee, Ra);
        __builtin_amdgcn_sched_barrier(0);
        step(B, C, ee + 16, Rb);
        __builtin_amdgcn_sched_barrier(0);
        step(C, D, ee + 32, Rc);
        __builtin_amdgcn_sched_barrier(0);
        step(D, E, ee + 48, Rd);
        __builtin_amdgcn_sched_barrier(0);
        if (RANKS) {
            uint4 *const rq = reinterpret_cast<uint4 *>(rk + ee);
            rq[0] = Ra; rq[1] = Rb; rq[2] = Rc; rq[3] = Rd;
        }
    };
    uint4 G0 = ld(0), G1 = ld(1), G2 = ld(2), G3 = ld(3), G4 = ld(4);
    uint64_t e = e0, gi = 0;
    // 128 elements a round, their 8 granules (128 B of the tile) loaded together a round ahead:
    // a lane's loads are 4 KiB from its neighbours', so with 4 granules a round each line was
    // loaded in two halves a round apart, and the wave's 64 lines were gone from L2 in between
    // (the walk read 2.7x its input from HBM, profiles/r4f_nyb_adaptive_pmc.txt)
    for (; e + 128 <= e1; e += 128, gi += 8) {
        const uint4 N1 = ld(gi + 5), N2 = ld(gi + 6), N3 = ld(gi + 7), N4 = ld(gi + 8);
        const uint4 N5 = ld(gi + 9), N6 = ld(gi + 10), N7 = ld(gi + 11), N8 = ld(gi + 12);
        quad(G0, G1, G2, G3, G4, e);
        quad(G4, N1, N2, N3, N4, e + 64);
        G0 = N4; G1 = N5; G2 = N6; G3 = N7; G4 = N8;
    }
    for (; e + 64 <= e1; e += 64, gi += 4) {
        const uint4 N1 = ld(gi + 5), N2 = ld(gi + 6), N3 = ld(gi + 7), N4 = ld(gi + 8);
        quad(G0, G1, G2, G3, G4, e);
        G0 = G4; G1 = N1; G2 = N2; G3 = N3; G4 = N4;
    }
    for (; e < e1; e += 16) {   // the last tile's ragged end, 16 elements at a time
        const uint32_t nk = e1 - e < 16 ? (uint32_t)(e1 - e) : 16u;
        const uint32_t pv = (cc << 3);
        uint32_t R[4] = {~0u, ~0u, ~0u, ~0u}, X[4] = {0u, 0u, 0u, 0u};
        for (uint32_t k = 0; k < nk; ++k) {
            const uint32_t x = in[e + 1 + k];
            uint32_t pb;
            bool hit;
            const uint64_t L2 = mtf_touch8(Lc, x, pb, hit);
            s_L[cc][t] = L2;
            const uint32_t r = hit ? pb >> 3 : (Lc >> 56) == 0ull ? 0xFEu : 0xFFu;
            if (RANKS) rk[e + k] = (uint8_t)r;
            R[k >> 2] = (R[k >> 2] & ~(255u << (8 * (k & 3)))) | (r << (8 * (k & 3)));
            X[k >> 2] |= x << (8 * (k & 3));
            anyz |= x == 0u ? 0x80u : 0u;
            cc = (x >> 3) & 15u;
            Lc = s_L[cc][t];
        }
        if (RANKS) post(R, X, pv, e, (1u << nk) - 1u);
    }
    uint64_t cnts = 0;   // nibble c = entries of list c
    if (anyz) {
        // a zero byte makes the pads ambiguous: the tile again, with counts (rare on text)
        for (int c = 0; c < 16; ++c) s_L[c][t] = 0ull;
        accp = FSMP_ID;
        nrec = 0;
        uint32_t pvb = prev0;
        for (uint64_t f = e0; f < e1; f += 16) {
            const uint32_t nk = e1 - f < 16 ? (uint32_t)(e1 - f) : 16u;
            const uint32_t pv = pvb;
            uint32_t R[4] = {~0u, ~0u, ~0u, ~0u}, X[4] = {0u, 0u, 0u, 0u};
            for (uint32_t k = 0; k < nk; ++k) {
                const uint32_t x = in[f + 1 + k], c = (pvb >> 3) & 15u;
                uint64_t L = s_L[c][t];
                uint32_t n = (uint32_t)(cnts >> (4 * c)) & 15u;
                const uint32_t nb = n;
                const int r0 = mtf_touch64(L, n, x);
                s_L[c][t] = L;
                cnts = (cnts & ~(15ull << (4 * c))) | ((uint64_t)n << (4 * c));
                const uint32_t r = r0 >= 0 ? (uint32_t)r0 : nb < 8 ? 0xFEu : 0xFFu;
                if (RANKS) rk[f + k] = (uint8_t)r;
                R[k >> 2] = (R[k >> 2] & ~(255u << (8 * (k & 3)))) | (r << (8 * (k & 3)));
                X[k >> 2] |= x << (8 * (k & 3));
                pvb = x;
            }
            if (RANKS) post(R, X, pv, f, (1u << nk) - 1u);
        }
    }
    if (RANKS) head[tile] = make_uint2(nrec, accp);
    for (int c = 0; c < 16; ++c) {
        const uint64_t L = s_L[c][t];
        uint32_t nz = 0;   // zero bytes: the pads
#pragma unroll
        for (int q = 0; q < 8; ++q) nz += ((L >> (8 * q)) & 255u) == 0u ? 1u : 0u;
        summ[tile].L[c] = L;
        summ[tile].cnt[c] = (uint8_t)(anyz ? (uint32_t)(cnts >> (4 * c)) & 15u : 8u - nz);
    }
}

// k_mtf_resolve: the first touches of k_mtf_walk<2>'s step records, from each tile's entry
// lists, and the nybble encoder's tile summaries (-> fraw). The j-th first touch of context c in a
// tile (j < 8: the list held the j bytes touched in the tile above the entry list) has rank j +
// its position among the entry list's bytes not touched in the tile yet (a miss past 7, or when
// absent): G_c = the entry list less those bytes (LDS column t); each first touch takes its byte
// out. A record's second uint4 becomes the step's settled ranks at its first touches (the writer
// reads the tile's records into LDS; rank bytes scattered into rk cost 0.37 ms per GiB in
// partial-line writes), and rk gets the tile's last element (read across the tile boundary). One
// lane per tile.
__global__ __launch_bounds__(256) void k_mtf_resolve(uint64_t len, uint64_t ntiles, const MtfSum *__restrict__ entry,
                                                     uint4 *__restrict__ rec, const uint2 *__restrict__ head,
                                                     uint8_t *__restrict__ rk, uint4 *__restrict__ fraw,
                                                     uint4 *__restrict__ fsumm)
{
    __shared__ uint64_t s_G[16][256];
    const int t = threadIdx.x;
    const uint64_t tile = (uint64_t)blockIdx.x * 256 + t;
    if (tile >= ntiles) return;   // no barriers below
    const uint2 hd = head[tile];
    uint64_t jn = 0, gv = 0;   // nibble c: first touches so far / bytes left in G_c
    for (int c = 0; c < 16; ++c) {
        s_G[c][t] = entry[tile].L[c];
        gv |= (uint64_t)min((uint32_t)entry[tile].cnt[c], 8u) << (4 * c);
    }
    uint4 *const trec = rec + 2 * tile * MTF_REC;
    const uint64_t e0 = tile * MTF_TILE;
    const uint32_t last = (uint32_t)(((e0 + MTF_TILE < len - 1) ? e0 + MTF_TILE : len - 1) - e0 - 1);   // the tile's last element
    uint32_t accp = FSMP_ID;
    // records 4 at a time, the next 4 in flight (the first 4 slots read before the count is
    // known: they exist for every tile; one record at a time made each a dependent round trip)
    uint4 A[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) A[k] = trec[k];
    for (uint32_t i0 = 0; i0 < hd.x; i0 += 4) {
      uint4 B[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) B[k] = (i0 + 4 + (uint32_t)(k >> 1) < hd.x) ? trec[2 * i0 + 8 + k] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const uint32_t i = i0 + (uint32_t)kk;
        if (i >= hd.x) break;
        const uint4 q0 = A[2 * kk], q1 = A[2 * kk + 1];
        const uint32_t X[4] = {q1.x, q1.y, q1.z, q1.w};
        uint32_t P[4] = {0u, 0u, 0u, 0u}, H = q0.y & 0xFFFFu, F = q0.y >> 16;
        const uint32_t step = q0.z & 255u, pv = (q0.z >> 8) & 255u, nk = q0.z >> 16;
        accp = fsmp_then(accp, q0.x);
        while (F) {
            const uint32_t k = (uint32_t)__builtin_ctz(F);
            F &= F - 1u;
            const uint32_t x = (X[k >> 2] >> (8 * (k & 3))) & 255u;
            const uint32_t p = k ? (X[(k - 1) >> 2] >> (8 * ((k - 1) & 3))) & 255u : pv;
            const uint32_t c = (p >> 3) & 15u;
            const uint32_t j = (uint32_t)(jn >> (4 * c)) & 15u, v = (uint32_t)(gv >> (4 * c)) & 15u;
            uint32_t rank = 0xFFu;
            if (j < 8u) {
                const uint64_t G = s_G[c][t];
                const uint64_t tt = G ^ (0x0101010101010101ull * x);
                const uint64_t z = (tt - 0x0101010101010101ull) & ~tt & 0x8080808080808080ull;
                const uint32_t pos = z ? (uint32_t)__builtin_ctzll(z) >> 3 : 8u;
                if (pos < v) {
                    rank = j + pos <= 7u ? j + pos : 0xFFu;
                    const uint64_t lowm = (1ull << (8 * pos)) - 1ull;   // out: the bytes above come down
                    s_G[c][t] = (G & lowm) | ((G >> 8) & ~lowm);
                    gv -= 1ull << (4 * c);
                }
                jn += 1ull << (4 * c);
            }
            P[k >> 2] |= rank << (8 * (k & 3));
            H |= (rank != 0xFFu ? 1u : 0u) << k;
            if (16 * step + k == last) rk[e0 + last] = (uint8_t)rank;
        }
        accp = fsmp_then(accp, fsmp(nyb_lane_fsm<M_NYB_ENC>(H, 0u, nk >= 16 ? 0xFFFFu : (1u << nk) - 1u)));
        trec[2 * i + 1] = make_uint4(P[0], P[1], P[2], P[3]);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) A[k] = B[k];
    }
    const uint4 f = fsm_pack(fsmp_unpack(fsmp_then(accp, hd.y)));
    fraw[tile] = f;    // kept for a later write pass (a shard body's: its plan's scan rewrites fsumm)
    fsumm[tile] = f;   // the transducer's tile summaries, ready for its scan
}

// parent[g] = composition of child summaries [64 g, 64 g + 64); one lane per (group, context)
__global__ __launch_bounds__(256) void k_mtf_reduce(const MtfSum *__restrict__ child, uint64_t nchild,
                                                    MtfSum *__restrict__ parent)
{
    const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t g = id >> 4;
    const int c = (int)(id & 15);
    if (g * MTF_FAN >= nchild) return;
    uint64_t L = 0;
    uint32_t n = 0;
    const uint64_t k1 = (g + 1) * MTF_FAN < nchild ? (g + 1) * MTF_FAN : nchild;
    for (uint64_t k0 = g * MTF_FAN; k0 < k1; k0 += 8) {   // 8 children's loads in flight
        uint64_t Ls[8];
        uint32_t ns[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            Ls[q] = k0 + q < k1 ? child[k0 + q].L[c] : 0ull;
            ns[q] = k0 + q < k1 ? child[k0 + q].cnt[c] : 0u;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) mtf_apply(L, n, Ls[q], ns[q]);
    }
    parent[g].L[c] = L;
    parent[g].cnt[c] = (uint8_t)n;
}

// child_entry[k] for the children of group g, from parent_entry[g]; the state after the
// last child of the last group goes to *final (optional)
__global__ __launch_bounds__(256) void k_mtf_down(const MtfSum *__restrict__ child, uint64_t nchild,
                                                  const MtfSum *__restrict__ parent_entry,
                                                  MtfSum *__restrict__ child_entry, MtfSum *__restrict__ final_state)
{
    const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t g = id >> 4;
    const int c = (int)(id & 15);
    if (g * MTF_FAN >= nchild) return;
    uint64_t L = parent_entry[g].L[c];
    uint32_t n = parent_entry[g].cnt[c];
    const uint64_t k1 = (g + 1) * MTF_FAN < nchild ? (g + 1) * MTF_FAN : nchild;
    for (uint64_t k0 = g * MTF_FAN; k0 < k1; k0 += 8) {   // 8 children's loads in flight
        uint64_t Ls[8];
        uint32_t ns[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            Ls[q] = k0 + q < k1 ? child[k0 + q].L[c] : 0ull;
            ns[q] = k0 + q < k1 ? child[k0 + q].cnt[c] : 0u;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if (k0 + q < k1) {
                child_entry[k0 + q].L[c] = L;
                child_entry[k0 + q].cnt[c] = (uint8_t)n;
            }
            mtf_apply(L, n, Ls[q], ns[q]);
        }
    }
    if (final_state && k1 == nchild) {
        final_state->L[c] = L;
        final_state->cnt[c] = (uint8_t)n;
    }
}

// ------------------------------------------------------------------------------------
// Chunked nybble container "DCNK" (SURVEY.md §8(e) "adaptive decode needs independent-chunk
// framing", §8(f)4): the input is cut into chunks of K bytes and each chunk is stored as the
// reference's own stream of that chunk (compress_bytestring on the chunk: header, packed
// nybbles, LITERAL fallback), so every chunk decodes alone with decompress_bytestring.
// Layout: u32 magic 'DCNK', u32 version 1, u32 modify, u32 K, u64 n, u64 nchunks,
// u64 off[nchunks + 1] (chunk streams, relative to the payload), payload.
// One lane walks one chunk (the adaptive lists are sequential within a chunk); the lists
// live in LDS as u64 words, one column per lane.
// ------------------------------------------------------------------------------------
#define NYBK_MAGIC 0x4B4E4344u   // "DCNK"
#define NYBK_HEAD 32

static __device__ __forceinline__ uint64_t mtf_init_word()
{
    return 0x736E696F61746520ull;   // " etaoins", byte k = entry k
}

// Adaptive decode of one stream (decompress_bytestring with modify, :734-817): every byte
// depends on the lists as every byte before it left them, so one wave walks the stream with
// all state on the chip and nothing on the loop's dependency chain touching memory:
//   * the 16 move-to-front lists as u64 words in VGPR lanes 0..15 (v_readlane /
//     v_writelane by the uniform context index), touched with 64-bit scalar bit operations;
//   * the input as two 256-B windows in one VGPR each (lane j = dword j), the next window's
//     load issued 256 bytes before it is needed;
//   * the output accumulated a dword at a time into a 256-B VGPR window (lane j = dword j)
//     and stored whole, bytes outside [out, out + written) left untouched.
// (The single-lane loop it replaces read in[pos] and out[o - 1] from global memory on every
// byte: two dependent round trips per output byte.)
// lane `lane` (uniform) of dst := val (uniform): a compare and a select (v_writelane_b32 needs
// its lane index in M0 on gfx9 when the value is an SGPR)
static __device__ __forceinline__ uint32_t writelane(uint32_t dst, uint32_t val, uint32_t lane)
{
    return (threadIdx.x & 63) == lane ? val : dst;
}

static __device__ __forceinline__ uint32_t adec_load(uintptr_t A, uintptr_t lo, uintptr_t hi, int lane)
{
    const uintptr_t ad = A + 4 * (uintptr_t)lane;
    return (ad + 4 > lo && ad < hi) ? *reinterpret_cast<const uint32_t *>(ad) : 0u;
}

// store the output window (lane j = dword OA + 4j) restricted to bytes [lo, hi)
static __device__ __forceinline__ void adec_flush(uint32_t w, uintptr_t OA, uintptr_t lo, uintptr_t hi, int lane)
{
    const uintptr_t ad = OA + 4 * (uintptr_t)lane;
    if (ad >= lo && ad + 4 <= hi) {
        *reinterpret_cast<uint32_t *>(ad) = w;
    } else {
        for (int k = 0; k < 4; ++k)
            if (ad + k >= lo && ad + k < hi) *reinterpret_cast<uint8_t *>(ad + k) = (uint8_t)(w >> (8 * k));
    }
}

// Adaptive decode, second form (the product path): two passes.
//  1. The token structure of a nybble stream does not depend on the lists: a nybble with its
//     high bit set is a hit (rank = its low 3 bits), any other starts a 2-nybble literal. So
//     the static decoder's transducer kernels (k_fsm_*<M_NYB_DEC>, parallel) write one token
//     byte per output byte straight into the output buffer: the literal itself (always < 0x80)
//     or 0x80 | rank (FsmAux.tokens), after out[0] = in[1].
//  2. k_nyb_resolve, one wave, replaces every token in place by its byte. The sequential loop
//     holds no parsing: per byte, the list of the context of the byte before is read from VGPR
//     lane c (v_readlane), touched with 64-bit scalar operations (a hit's rank is its position,
//     a literal's position is found by a SWAR zero-byte test), and written back (v_writelane).
//     Tokens arrive by scalar loads one 64-byte block ahead; the 64 bytes of a block are
//     assembled in SGPRs at static positions (the loop is unrolled over the block) and leave
//     as 16 dwords of one VGPR.

typedef __attribute__((address_space(4))) const uint32_t c_u32;   // scalar (s_load) reads
typedef uint32_t u32x32 __attribute__((ext_vector_type(32)));   // the 16 lists as 32 SGPR dwords



// Fourth form (the product path since r3b): what a token gives without the lists is
// computed beforehand, in parallel (k_nyb_adec_ctl, one dword per token), and the sequential
// step is scalar instructions on the 16 lists in s[64:95]: the list by M0 from the byte
// before (s_bfe of its bits 2..6: M0 = 2c + a don't-care bit the 64-bit s_movrels ignores,
// tools/ubench/movrels.hip); a hit's byte by one s_bfe_u64 of the list (width 8 at 8p); the
// move to front by the mask of the bytes past p. A literal still needs update_context's
// search (:674-682): the encoder writes a pending hit raw when a miss follows it, so a
// literal can be in its list (the r3 tokens showed it at 1 in ~30 symbols of the bench text).
// Literals take the search on a uniform branch: 26 scalar instructions; hits 15
// (k_nyb_resolve_s's form: 28 for every byte).
// ctl[i] for the token at out position k0 + i: bits 5:0 the S_BFE_U64 offset 8p (56 for a
// literal), bits 22:16 its width (8 for a hit, 0 for a literal), bit 23 the search, bits
// 31:24 the literal.
__global__ __launch_bounds__(256) void k_nyb_adec_ctl(const uint8_t *__restrict__ tok, uint64_t k0, uint64_t k1,
                                                      uint64_t n, uint32_t *__restrict__ ctl)
{
    for (uint64_t i = k0 + (uint64_t)blockIdx.x * 256 + threadIdx.x; i < k1; i += (uint64_t)gridDim.x * 256) {
        const uint32_t t = tok[i];
        // bit 23 (outside the S_BFE_U64 fields): a literal, whose position the step searches.
        // (Only a literal followed by a literal or ending the stream can be a flushed hit when
        // the stream is the encoder's, and skipping the others' search measured 6% faster on
        // 4 MiB of text; but a stream whose input held bytes >= 0x80 desynchronises the lists
        // (the golden nybble vectors have one), and a check for that costs a re-encode.)
        (void)n;
        ctl[i - k0] = (t & 0x80u) ? (0x80000u | (8u * (t & 7u))) : ((t << 24) | 56u | 0x800000u);
    }
}

// STEP_C_ASM(W): the step's text; W is inserted right after the join, where v is final (the
// block loop puts v_writelane there: issued after the s_movreld it drew a compiler s_nop)
#define STEP_C_ASM_X(W, V, VP, C, SFX)                                                                         \
        "s_lshr_b32 %[" V "], %[" C "], 24\n\t"                /* the literal (0 for a hit); first, so   \
                                                          the previous s_movreld is not followed \
                                                          by an M0 write (a compiler s_nop) */  \
        "s_bfe_u32 m0, %[" VP "], 0x50002\n\t"             /* 2c (+ bit 2 of the byte: ignored) */  \
        "s_bitcmp1_b32 %[" C "], 23\n\t"                   /* a literal: search its position */     \
        "s_movrels_b64 s[96:97], s[64:65]\n\t"          /* L = the list of context c */          \
        "s_cbranch_scc0 .Lhit%=" SFX "\n\t"                                                           \
        "s_mul_i32 s98, %[" V "], 0x1010101\n\t"           /* (update_context's search :674-682) */ \
        "s_xor_b32 s99, s98, s97\n\t"                                                          \
        "s_xor_b32 s98, s98, s96\n\t"                                                          \
        "s_sub_u32 %[T], s98, 0x1010101\n\t"                                                   \
        "s_andn2_b32 %[T], %[T], s98\n\t"                                                      \
        "s_and_b32 s98, %[T], 0x80808080\n\t"          /* zero bytes of the low half */         \
        "s_sub_u32 %[T], s99, 0x1010101\n\t"                                                   \
        "s_andn2_b32 %[T], %[T], s99\n\t"                                                      \
        "s_and_b32 s99, %[T], 0x80808080\n\t"                                                  \
        "s_ff1_i32_b64 %[T], s[98:99]\n\t"                                                     \
        "s_lshr_b32 %[T], %[T], 3\n\t"                                                         \
        "s_min_u32 %[T], %[T], 7\n\t"                  /* absent: 7, the last entry drops */    \
        "s_lshl_b32 %[T], %[T], 3\n\t"                                                         \
        "s_lshl_b64 %[N], -1, %[T]\n\t"                                                        \
        "s_branch .Ljoin%=" SFX "\n"                                                                  \
        ".Lhit%=" SFX ":\n\t"                                                                         \
        "s_bfe_u64 s[98:99], s[96:97], %[" C "]\n\t"       /* a hit: the byte at its rank */        \
        "s_or_b32 %[" V "], %[" V "], s98\n\t"                                                         \
        "s_lshl_b64 %[N], -1, %[" C "]\n"                                                          \
        ".Ljoin%=" SFX ":\n\t"                                                                        \
        W                                                                                      \
        "s_lshl_b64 %[N], %[N], 8\n\t"                 /* the bytes past p (they stay) */       \
        "s_lshl_b64 s[98:99], s[96:97], 8\n\t"                                                 \
        "s_andn2_b64 s[98:99], s[98:99], %[N]\n\t"     /* bytes 0..p-1 move up one */           \
        "s_and_b64 s[96:97], s[96:97], %[N]\n\t"                                               \
        "s_or_b64 s[96:97], s[96:97], s[98:99]\n\t"                                            \
        "s_or_b32 s96, s96, %[" V "]\n\t"                  /* v to the front (:665-687) */          \
        "s_movreld_b64 s[64:65], s[96:97]"

#define STEP_C_ASM(W) STEP_C_ASM_X(W, "v", "vp", "c", "")

// M0 is compiler-reserved: an "m0" clobber is not honoured (hipcc warns that reserved
// registers on the clobber list may not be preserved), so every statement that writes M0
// saves it on entry and restores it before it ends (cdna_hip_programming.md §5.7): whatever
// the compiler keeps in M0 survives the statement
#define M0_SAVE "s_mov_b32 %[m0keep], m0\n\t"
#define M0_RESTORE "\n\ts_mov_b32 m0, %[m0keep]"
static __device__ __forceinline__ uint32_t adec_step_c(u32x32 &lists, uint32_t &vprev, uint32_t c)
{
    uint32_t v, T, m0keep;
    uint64_t N;   // (compiler-chosen scratch; the fixed pairs s96-s99 stay clear of s100-s101,
                  //  which gfx950 reserves)
    asm volatile(M0_SAVE STEP_C_ASM("") M0_RESTORE
        : [lists] "+{s[64:95]}"(lists), [v] "=&s"(v), [N] "=&s"(N), [T] "=&s"(T), [m0keep] "=&s"(m0keep)
        : [vp] "s"(vprev), [c] "s"(c)
        : "s96", "s97", "s98", "s99", "scc");
    vprev = v;
    return v;
}

// four steps in one statement (between two asm statements the compiler puts an s_nop: it
// cannot see that the next one's first instruction is no hazard after the s_movreld)
#define STEP_WL(V, KK) "v_writelane_b32 %[ov], %[" V "], %[" KK "]\n\t"
template <int K>
static __device__ __forceinline__ void adec_step_cw4(u32x32 &lists, uint32_t &vprev, const uint32_t *c, uint32_t &ov)
{
    uint32_t v0, v1, v2, v3, T, m0keep;
    uint64_t N;
    asm volatile(M0_SAVE
                 STEP_C_ASM_X(STEP_WL("v0", "k0"), "v0", "vp", "c0", "a") "\n\t"
                 STEP_C_ASM_X(STEP_WL("v1", "k1"), "v1", "v0", "c1", "b") "\n\t"
                 STEP_C_ASM_X(STEP_WL("v2", "k2"), "v2", "v1", "c2", "c") "\n\t"
                 STEP_C_ASM_X(STEP_WL("v3", "k3"), "v3", "v2", "c3", "d")
                 M0_RESTORE
        : [lists] "+{s[64:95]}"(lists), [v0] "=&s"(v0), [v1] "=&s"(v1), [v2] "=&s"(v2), [v3] "=&s"(v3),
          [N] "=&s"(N), [T] "=&s"(T), [ov] "+v"(ov), [m0keep] "=&s"(m0keep)
        : [vp] "s"(vprev), [c0] "s"(c[0]), [c1] "s"(c[1]), [c2] "s"(c[2]), [c3] "s"(c[3]),
          [k0] "i"(K), [k1] "i"(K + 1), [k2] "i"(K + 2), [k3] "i"(K + 3)
        : "s96", "s97", "s98", "s99", "scc");
    vprev = v3;
}


// a 64-token block: group G from A (loaded), group G + 1 into B while it runs (its load
// issued after the first steps' wait), and so on: G = 0, 2
template <int G>
static __device__ __forceinline__ void adec_block(u32x32 &lists, uint32_t &vprev, uint32_t (&A)[16], uint32_t (&B)[16],
                                                  c_u32 *blk, c_u32 *next_blk, uint32_t &ov)
{
    adec_step_cw4<16 * G>(lists, vprev, A, ov);
    asm volatile("" ::: "memory");   // group G + 1's load leaves after the wait for group G
#pragma unroll
    for (int q = 0; q < 16; ++q) B[q] = blk[16 * (G + 1) + q];
    adec_step_cw4<16 * G + 4>(lists, vprev, A + 4, ov);
    adec_step_cw4<16 * G + 8>(lists, vprev, A + 8, ov);
    adec_step_cw4<16 * G + 12>(lists, vprev, A + 12, ov);
    adec_step_cw4<16 * G + 16>(lists, vprev, B, ov);
    asm volatile("" ::: "memory");
    c_u32 *nx = (G + 2 < 4) ? blk + 16 * (G + 2) : next_blk;   // group G + 2, or the next block's first
#pragma unroll
    for (int q = 0; q < 16; ++q) A[q] = nx[q];
    adec_step_cw4<16 * G + 20>(lists, vprev, B + 4, ov);
    adec_step_cw4<16 * G + 24>(lists, vprev, B + 8, ov);
    adec_step_cw4<16 * G + 28>(lists, vprev, B + 12, ov);
    if (G == 0) adec_block<2>(lists, vprev, A, B, blk, next_blk, ov);
}

// one wave resolves the tokens of out[k0, k1) in place from ctl[0, k1 - k0); state[0..31] the
// 16 lists, state[32] the byte before k0 (first: the initial lists and out[k0 - 1])
__global__ __launch_bounds__(64) void k_nyb_resolve_c(uint8_t *__restrict__ out, uint64_t k0, uint64_t k1,
                                                      const uint32_t *__restrict__ ctl, uint32_t *__restrict__ state,
                                                      int first)
{
    const int lane = (int)threadIdx.x;
    u32x32 lists;
    uint32_t vprev;
    if (first) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            lists[2 * c] = (uint32_t)mtf_init_word();
            lists[2 * c + 1] = (uint32_t)(mtf_init_word() >> 32);
        }
        vprev = (uint32_t)__builtin_amdgcn_readfirstlane((int)out[k0 - 1]);
    } else {
        c_u32 *st = (c_u32 *)state;
#pragma unroll
        for (int q = 0; q < 32; ++q) lists[q] = st[q];
        vprev = st[32];
    }
    c_u32 *cw = (c_u32 *)ctl;
    const uint64_t m = k1 - k0, nfull = m / 64;
    if (nfull) {
        uint32_t A[16], B[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) A[q] = cw[q];
        for (uint64_t b = 0; b < nfull; ++b) {
            uint32_t ov = 0;   // lane k: the byte of token 64b + k
            c_u32 *blk = cw + 64 * b;
            adec_block<0>(lists, vprev, A, B, blk, (b + 1 < nfull) ? blk + 64 : blk, ov);
            out[k0 + 64 * b + lane] = (uint8_t)ov;
        }
    }
    uint32_t ov = 0;   // the last < 64 tokens, one at a time
    for (uint64_t i = 64 * nfull; i < m; ++i) {
        const uint32_t v = adec_step_c(lists, vprev, cw[i]);
        ov = (uint64_t)lane == i - 64 * nfull ? v : ov;
    }
    if ((uint64_t)lane < m - 64 * nfull) out[k0 + 64 * nfull + lane] = (uint8_t)ov;
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 32; ++q) state[q] = lists[q];
        state[32] = vprev;
    }
}



// ---- one lane per stream (DCNK chunks, dc_nyb_decompress_batch) ----------------------
// A lane walks its own stream byte by byte (the lists make every byte depend on the one
// before), and a launch has one wave per 64 streams: 4 waves per CU on 65536 streams of 4 KiB.
// r4's loops read in[pos] and wrote out[q] one byte at a time: a dependent global round trip
// per input byte (~1.4 us: 46.6 GB/s) and byte stores to 64 private lines per wave (22.7x the
// output in HBM writes). Here a lane's memory traffic moves only at IO points the whole wave
// reaches together, so no step of the byte loop waits on memory:
//  * input the lane reads exactly one byte per step of (the encoder, the length pass) is walked
//    in 16-B granules, 8 per round, the next round's 8 loads in flight (nl_walk);
//  * input the lane reads at its own rate (the decoder: 0.5-1 byte per output byte) sits in an
//    LDS ring of NL_RING bytes per lane, topped up 64 B at a time at the IO points, with the
//    next 64 B always in flight in registers (nyb_wave_decode);
//  * output gathers in an LDS ring of two 64-B lines per lane and leaves as whole lines (4 x
//    16 B) at the IO points; the line the stream shares with the bytes before it waits in LDS
//    and goes byte by byte at the end, with the last partial line (NlOut).
#define NL_RING 128    /* decoder input ring per lane (bytes): two 64-B blocks behind the one in flight */
#define NL_RSTR 144    /* its LDS row stride: 16-B aligned, lanes' rows 4 banks apart */
#define NL_LINE 128    /* output leaves in whole 128-B lines (64-B halves a point apart wrote 1.46x) */
#define NL_ORING 256   /* output ring per lane: the line being gathered and the next */
#define NL_OSTR 272
#define NL_P 32        /* decoder steps between two IO points (<= 32 bytes in, <= 32 out) */
__device__ uint4 nl_zero[1];   // the granule lanes without a stream read (never written)
// (granule pointers are formed as p - (p & 15), never through an integer: a pointer rebuilt from
// a uintptr_t made the compiler emit flat loads, which also count in lgkmcnt, so every LDS wait
// of the byte loop waited for the granules in flight)
static __device__ __forceinline__ uint4 nl_ld(const uint4 *p) { return *p; }

struct NlOut {        // a lane's output [b + sh, ...): b = the start rounded down to NL_LINE
    uint8_t *b;
    uint32_t sh;
    uint64_t S;       // next line to send (offset from b, a multiple of NL_LINE)
    uint8_t *ring;
};
static __device__ __forceinline__ void nl_out_init(NlOut &o, uint8_t *dst, uint8_t *ring)
{
    o.sh = (uint32_t)((uintptr_t)dst & (NL_LINE - 1));
    o.b = dst - o.sh;
    o.S = 0;
    o.ring = ring;
}
// W = offset from b past the last byte put: send the line it completed (one per point at most:
// <= 32 bytes are put between points). The stream's first line, which holds bytes before the
// stream, goes byte by byte (once per stream).
static __device__ __forceinline__ void nl_out_point(NlOut &o, uint64_t W)
{
    if (W >= o.S + NL_LINE) {
        const uint4 *src = reinterpret_cast<const uint4 *>(o.ring + (o.S & (NL_ORING - 1)));
        if (o.S < o.sh) {
            for (uint32_t a = o.sh; a < NL_LINE; ++a) o.b[a] = o.ring[a];
        } else {
            uint4 v[NL_LINE / 16];
#pragma unroll
            for (int k = 0; k < NL_LINE / 16; ++k) v[k] = src[k];
            uint4 *d = reinterpret_cast<uint4 *>(o.b + o.S);
#pragma unroll
            for (int k = 0; k < NL_LINE / 16; ++k) d[k] = v[k];
        }
        o.S += NL_LINE;
    }
}
static __device__ __forceinline__ void nl_out_finish(const NlOut &o, uint64_t W)
{
    for (uint64_t a = o.S > o.sh ? o.S : o.sh; a < W; ++a) o.b[a] = o.ring[a & (NL_ORING - 1)];
}

// Lockstep walk of bytes [lo, hi) of a lane's granules g (offsets from g; every lane of the
// wave calls it, lanes without bytes with g = nl_zero, lo = hi = 0): fn(byte, valid) per byte
// in order, point() after every granule. 8 granules a round, the next round's in flight.
template <class Fn, class Pt>
static __device__ __forceinline__ void nl_walk(const uint4 *g, uint64_t lo, uint64_t hi, Fn fn, Pt point)
{
    const uint64_t k0 = lo >> 4, k1 = hi > lo ? (hi - 1) >> 4 : k0;
    const bool any = hi > lo;
    uint4 G[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) G[j] = nl_ld(g + min(k0 + (uint64_t)j, k1));
    for (uint64_t k = k0; __ballot(any && k <= k1); k += 8) {
        uint4 N[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) N[j] = nl_ld(g + min(k + 8 + (uint64_t)j, k1));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int64_t base = (int64_t)(16 * (k + j));
            const int64_t vlo = (int64_t)lo - base, vhi = (any ? (int64_t)hi : 0) - base;   // valid bytes [vlo, vhi)
            const uint32_t w[4] = {G[j].x, G[j].y, G[j].z, G[j].w};
#pragma unroll
            for (int e = 0; e < 16; ++e) fn((w[e >> 2] >> (8 * (e & 3))) & 255u, e >= vlo && e < vhi);
            point();
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) G[j] = N[j];
    }
}

// DCNK encode: one lane per chunk of K bytes, nybble_compress of the chunk
// (compress_bytestring, nybble_compression.c:887-1038) into its scratch slot of K + 2 bytes
__global__ __launch_bounds__(64) void k_nyb_chunk_enc(const uint8_t *__restrict__ in, uint64_t n, uint32_t K,
                                                      uint64_t nchunks, int modify, uint8_t *__restrict__ scr,
                                                      uint64_t *__restrict__ lens)
{
    __shared__ uint64_t s_L[16][64];
    __shared__ __attribute__((aligned(16))) uint8_t s_out[64 * NL_OSTR];
    const int t = threadIdx.x;
    const uint64_t ch = (uint64_t)blockIdx.x * 64 + t;
    const bool live = ch < nchunks;
    const uint8_t *x = in + (live ? ch * K : 0);
    const uint64_t len = live ? ((n - ch * K < K) ? n - ch * K : K) : 0;
    uint8_t *const slot = scr + (live ? ch * ((uint64_t)K + 2) : 0);
    for (int c = 0; c < 16; ++c) s_L[c][t] = mtf_init_word();
    NlOut o;
    nl_out_init(o, slot, s_out + t * NL_OSTR);
    uint64_t q = 0;   // bytes put
    auto put = [&](uint32_t v) { o.ring[(o.sh + q) & (NL_ORING - 1)] = (uint8_t)v; ++q; };
    uint32_t prev = len ? x[0] : 0u;
    if (len) { put(0xAF); put(prev); }
    int half = 0;
    uint32_t hi = 0;   // pending high nybble (with its byte's value, for a later rewrite)
    const uintptr_t xa = (uintptr_t)x;
    const uint4 *g = len > 1 ? reinterpret_cast<const uint4 *>(x - (xa & 15)) : nl_zero;
    const uint64_t sh = len > 1 ? xa & 15 : 0;
    nl_walk(g, len > 1 ? sh + 1 : 0, len > 1 ? sh + len : 0,
        [&](uint32_t v, bool valid) {
            if (valid) {
                const uint32_t c = (prev >> 3) & 15u;
                uint32_t pb;
                bool hit;
                // compress_byte_index :833-839 (rank before the touch), update_context :665-687
                const uint64_t L = mtf_touch8(s_L[c][t], v, pb, hit);
                if (modify) s_L[c][t] = L;
                const int r = hit ? (int)(pb >> 3) : -1;
                if (r < 0) {
                    if (half) { put(prev); half = 0; }   // miss at offset 1 (:855-857)
                    put(v);
                } else if (!half) {
                    hi = (8u | (uint32_t)r) << 4;
                    half = 1;
                } else {
                    put(hi | 8u | (uint32_t)r);
                    half = 0;
                }
                prev = v;
            }
        },
        [&]() { nl_out_point(o, o.sh + q); });
    if (half) put(prev);   // odd tail (:1000-1009): the last byte raw
    if (live && q >= len) {   // LITERAL fallback (:1018-1037): the slot rewritten, byte by byte (rare)
        slot[0] = ' ';
        for (uint64_t i = 0; i < len; ++i) slot[1 + i] = x[i];
        q = len + 1;
    } else if (live) {
        nl_out_point(o, o.sh + q);
        nl_out_finish(o, o.sh + q);
    }
    if (live) lens[ch] = q;
}

// single workgroup: off[0..nchunks] = exclusive scan of lens (off[nchunks] = total)
__global__ __launch_bounds__(1024) void k_scan_u64(const uint64_t *__restrict__ lens, uint64_t count,
                                                   uint64_t *__restrict__ off)
{
    __shared__ uint64_t s[1024];
    const int t = threadIdx.x;
    const uint64_t per = (count + 1023) / 1024;
    const uint64_t a0 = (uint64_t)t * per, a1 = (a0 + per < count) ? a0 + per : count;
    uint64_t sum = 0;
    uint64_t k = a0;   // 8 loads in flight per round (one round trip per count made it latency-bound)
    for (; k + 8 <= a1; k += 8) {
        uint64_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = lens[k + j];
#pragma unroll
        for (int j = 0; j < 8; ++j) sum += v[j];
    }
    for (; k < a1; ++k) sum += lens[k];
    s[t] = sum;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const uint64_t v = t >= d ? s[t - d] : 0;
        __syncthreads();
        s[t] += v;
        __syncthreads();
    }
    uint64_t o = t ? s[t - 1] : 0;
    for (k = a0; k + 8 <= a1; k += 8) {
        uint64_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = lens[k + j];
#pragma unroll
        for (int j = 0; j < 8; ++j) { off[k + j] = o; o += v[j]; }
    }
    for (; k < a1; ++k) { off[k] = o; o += lens[k]; }
    if (t == 1023) off[count] = s[1023];
}

// one workgroup per chunk: scratch stream -> payload
__global__ __launch_bounds__(256) void k_nyb_chunk_copy(const uint8_t *__restrict__ scr, uint32_t K,
                                                        const uint64_t *__restrict__ off, uint8_t *__restrict__ payload)
{
    const uint64_t ch = blockIdx.x;
    const uint8_t *src = scr + ch * ((uint64_t)K + 2);
    const uint64_t a = off[ch], len = off[ch + 1] - a;
    for (uint64_t i = threadIdx.x; i < len; i += 256) payload[a + i] = src[i];
}

// One lane decodes one whole reference stream (decompress_bytestring, nybble_compression.c:
// 734-817) of m bytes at src into exactly `expect` bytes at o (every lane of the wave calls
// it; lanes without a stream pass live = false). Type dispatch (:744, :799, :806): 0xAF
// nybbles, ' ' the raw bytes after it, any other type byte (any_type; DCNK chunks are never
// written so) every byte including the type byte. Returns false when the stream does not
// decode to `expect` bytes. One output byte per step: the raw byte 1 of a nybble stream, then
// a token each (a nybble with bit 3 set: a hit, its rank; any other: a literal of 2 nybbles).
static __device__ __forceinline__ bool nyb_wave_decode(const uint8_t *__restrict__ src, uint64_t m, uint64_t expect, int modify,
                                       bool any_type, uint8_t *__restrict__ o, bool live, uint64_t (*sL)[64],
                                       uint8_t *ring, uint8_t *oring, int t)
{
    if (!live) m = 0;
    // the input ring: ring[F - NL_RING, F) holds the stream's bytes from offset F - NL_RING of g
    // (16-B granules, the stream's first byte at offset sh), the 64 B at F in flight in r0..r3
    const uintptr_t sa = (uintptr_t)src;
    const uint32_t sh = m ? (uint32_t)(sa & 15) : 0u;
    const uint4 *const g = m ? reinterpret_cast<const uint4 *>(src - (sa & 15)) : nl_zero;
    const uint64_t gl = m ? (sh + m - 1) >> 4 : 0;
#pragma unroll
    for (int j = 0; j < NL_RING / 16; ++j) reinterpret_cast<uint4 *>(ring)[j] = nl_ld(g + min((uint64_t)j, gl));
    uint64_t F = NL_RING;
    constexpr uint64_t f0 = NL_RING / 16;
    uint4 r0 = nl_ld(g + min(f0, gl)), r1 = nl_ld(g + min(f0 + 1, gl)), r2 = nl_ld(g + min(f0 + 2, gl)),
          r3 = nl_ld(g + min(f0 + 3, gl));
    const uint32_t type = m ? ring[sh] : 0u;
    const bool raw = type != 0xAFu;
    bool ok = live;
    if (live) {
        if (m == 0) ok = expect == 0;
        else if (raw) ok = (type == ' ' || any_type) && m - (type == ' ' ? 1 : 0) == expect;
        else ok = m >= 2 ? expect != 0 : expect == 0;
    }
    const uint64_t qe = ok && m >= (raw ? 1u : 2u) ? expect : 0;   // bytes to write
    if (!raw)
        for (int c = 0; c < 16; ++c) sL[c][t] = mtf_init_word();
    uint64_t pos = sh + (raw ? (type == ' ' ? 1u : 0u) : 1u);   // offset (from g) of the next byte
    const uint64_t pe = sh + m;
    NlOut out;
    nl_out_init(out, o, oring);
    uint64_t q = 0;
    uint32_t prev = 0;
    int offn = 0;
    while (__ballot(q < qe)) {
        for (int i = 0; i < NL_P; ++i) {
            if (q < qe) {
                const uint32_t b0 = ring[pos & (NL_RING - 1)], b1 = ring[(pos + 1) & (NL_RING - 1)];
                uint32_t v = b0, adv = 2;   // raw byte (and a nybble stream's byte 1)
                if (!raw && q > 0) {
                    ok = ok && pos < pe;   // (tokens ran out before expect bytes)
                    const uint32_t nyb = offn ? b0 & 15u : b0 >> 4;
                    const uint32_t nxt = offn ? (pos + 1 < pe ? b1 >> 4 : 0u) : b0 & 15u;
                    const uint32_t c = (prev >> 3) & 15u;
                    const uint64_t L = sL[c][t];
                    if (nyb & 8u) { v = (uint32_t)(L >> (8 * (nyb & 7u))) & 255u; adv = 1; }
                    else { v = ((nyb & 7u) << 4) + nxt; adv = 2; }
                    if (modify) { uint32_t pb; bool hit; sL[c][t] = mtf_touch8(L, v, pb, hit); }
                }
                oring[(out.sh + q) & (NL_ORING - 1)] = (uint8_t)v;
                ++q;
                prev = v;
                offn += (int)adv;
                if (offn >= 2) { ++pos; offn -= 2; }
            }
        }
        // top the ring up while it leaves room (the bytes below pos are done with), and start the
        // next 64 B (pos moves <= NL_P bytes between points: F - pos stays >= 2, and a block is
        // written over bytes below pos only)
        if (F - pos <= NL_RING - 64) {
            uint4 *d = reinterpret_cast<uint4 *>(ring + (F & (NL_RING - 1)));
            d[0] = r0; d[1] = r1; d[2] = r2; d[3] = r3;
            F += 64;
            const uint64_t k = F >> 4;
            r0 = nl_ld(g + min(k, gl));
            r1 = nl_ld(g + min(k + 1, gl));
            r2 = nl_ld(g + min(k + 2, gl));
            r3 = nl_ld(g + min(k + 3, gl));
        }
        nl_out_point(out, out.sh + q);
    }
    if (!raw && pos < pe) ok = false;   // tokens past expect bytes
    nl_out_finish(out, out.sh + q);
    return ok;
}

// DCNK decode: one lane per chunk, its stream into out + ch*K; a stream that is not a
// nybble/LITERAL stream of exactly the chunk's length sets *err (bytes >= 0x80 do not
// round-trip through the reference codec, P8)
__global__ __launch_bounds__(64) void k_nyb_chunk_dec(const uint8_t *__restrict__ payload,
                                                      const uint64_t *__restrict__ off, uint64_t total, uint64_t n,
                                                      uint32_t K, uint64_t nchunks, int modify,
                                                      uint8_t *__restrict__ out, uint64_t *__restrict__ err)
{
    __shared__ uint64_t s_L[16][64];
    __shared__ __attribute__((aligned(16))) uint8_t s_in[64 * NL_RSTR];
    __shared__ __attribute__((aligned(16))) uint8_t s_out[64 * NL_OSTR];
    const int t = threadIdx.x;
    const uint64_t ch = (uint64_t)blockIdx.x * 64 + t;
    bool live = ch < nchunks;
    const uint64_t a = live ? off[ch] : 0, b = live ? off[ch + 1] : 0;
    const uint64_t expect = live ? ((n - ch * K < K) ? n - ch * K : K) : 0;
    if (live && (b < a || b > total || b - a < 1)) { *err = 1; live = false; }
    const bool ok = nyb_wave_decode(payload + a, live ? b - a : 0, expect, modify, false, out + (live ? ch * K : 0),
                                    live, s_L, s_in + t * NL_RSTR, s_out + t * NL_OSTR, t);
    if (live && !ok) *err = 1;
}

// dc_nyb_decompress_batch: the output length of each stream (one lane per stream): the token
// count of a 0xAF stream plus its first byte (the token structure needs no lists: a nybble with
// bit 3 set is a 1-nybble hit, any other starts a 2-nybble literal), the bytes after a ' ', or
// every byte under another type byte; an invalid range (end before start) counts 0 and flags err
__global__ __launch_bounds__(64) void k_nyb_batch_len(const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off,
                                                      uint64_t count, uint64_t *__restrict__ len, uint64_t *__restrict__ err)
{
    const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    const bool live = i < count;
    const uint64_t a = live ? in_off[i] : 0, b = live ? in_off[i + 1] : 0;
    if (live && b < a) *err = 1;
    const uint64_t m = live && b >= a ? b - a : 0;
    const uint32_t type = m ? in[a] : 0u;
    const bool nyb = m >= 3 && type == 0xAFu;   // tokens after byte 1
    // the token structure, 2 states per nybble (s = 1: the second nybble of a literal is next):
    // per byte, with h / l its nybbles' bit 3: tokens += s ? 1 : 1 + h, s' = s ? !l : h & !l
    uint64_t tok = 0;
    uint32_t st = 0;
    const uintptr_t sa = (uintptr_t)(in + a);
    const uint4 *g = nyb ? reinterpret_cast<const uint4 *>(in + a - (sa & 15)) : nl_zero;
    const uint64_t sh = nyb ? sa & 15 : 0;
    nl_walk(g, nyb ? sh + 2 : 0, nyb ? sh + m : 0,
        [&](uint32_t v, bool valid) {
            const uint32_t h = (v >> 7) & 1u, l = (v >> 3) & 1u;
            const uint32_t add = st ? 1u : 1u + h, ns = st ? l ^ 1u : h & (l ^ 1u);
            tok += valid ? add : 0u;
            st = valid ? ns : st;
        },
        []() {});
    uint64_t q = 0;
    if (m > 0) q = type == 0xAFu ? (m >= 2 ? 1 + tok : 0) : type == ' ' ? m - 1 : m;
    if (live) len[i] = q;
}

__global__ __launch_bounds__(64) void k_nyb_batch_dec(const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off,
                                                      const uint64_t *__restrict__ out_off, uint64_t count, int modify,
                                                      uint8_t *__restrict__ out, uint64_t *__restrict__ err)
{
    __shared__ uint64_t s_L[16][64];
    __shared__ __attribute__((aligned(16))) uint8_t s_in[64 * NL_RSTR];
    __shared__ __attribute__((aligned(16))) uint8_t s_out[64 * NL_OSTR];
    const int t = threadIdx.x;
    const uint64_t i = (uint64_t)blockIdx.x * 64 + t;
    bool live = i < count;
    const uint64_t a = live ? in_off[i] : 0, b = live ? in_off[i + 1] : 0;
    live = live && b >= a;   // (flagged by k_nyb_batch_len)
    const uint64_t o0 = live ? out_off[i] : 0, o1 = live ? out_off[i + 1] : 0;
    const bool ok = nyb_wave_decode(in + a, live ? b - a : 0, o1 - o0, modify, true, out + o0, live, s_L,
                                    s_in + t * NL_RSTR, s_out + t * NL_OSTR, t);
    if (live && !ok) *err = 1;
}

// ------------------------------------------------------------------------------------
// HBM copy probe (bench.py's reference rate, MI355X_MICROARCH.md's float4 copy): 16-B loads
// and stores with the nt hint, one uint4 per lane and one workgroup per 4 KiB (the full grid:
// 262144 workgroups on 1 GiB). r4 shapes (tools/ubench/copy_shapes.hip,
// profiles/r4a_copy_shapes.log): this shape 6.34 TB/s; grid-striding 4096-32768 workgroups
// with one uint4 per lane and step 4.57-4.69 (r3's probe, 16384, read 5.40 in the bench);
// 4 uint4 per lane and step at 32768 workgroups 6.24
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_copy_probe(const uint4 *__restrict__ src, uint4 *__restrict__ dst, uint64_t n16)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i < n16; i += stride) st_nt(dst + i, ld_nt(src + i));
}

#ifdef DC_AB_KERNELS
#include "dc_ab_kernels.inc"
#endif

// =====================================================================================
// host side
// =====================================================================================
#define DC_MAX_EVENTS 1024   /* HIP-event pairs per timing window (a C5 step launches ~40 kernels) */

struct dc_ctx {
    int device;
    hipStream_t stream;
    bool own_stream;
    // workspace
    uint16_t *d_bh;         size_t bh_cap;        // block histograms (u16 x 256 per block)
    uint64_t *d_off;        size_t off_cap;       // nblocks + 1
    uint32_t *d_plan;       size_t plan_cap;      // plan: per-block local offsets + workgroup totals
    uint64_t *d_msym;       size_t msym_cap;      // C5 fused front-end: first symbol index per block (+ total)
    uint32_t *d_gexp;       size_t gexp_cap;      // C5 decode: symbols >= 0x80 per group (dc_small_huff_decode)
    int *d_err;                                   // [8] text parse
    // error flags of plan/pack and of decode in rotating slots (32 x 4 ints each): every call
    // takes the next slot, which a kernel of the call before cleared (no memset launch)
    int *d_errp, *d_errd;
    uint32_t gen_p, gen_d;
    const dc_dtable *dec_fresh;                   // decoder tables current: this context's last pack built them,
    uint64_t dec_fresh_gen;                       // ... while g_table_gen had this value (see table_written)
    uint32_t *d_queue;                            // decode tuple scheduler heads (D8Sched)
    uint32_t *d_fix;        size_t fix_cap;       // decode redo: a u64 chunk mask per group
    uint32_t *d_fixpos;     size_t fixpos_cap;    // decode redo: bit offset of a flagged chunk
    uint64_t last_groups;                         // groups of the last S = 64 decode (redo mask length)
    uint64_t *d_hloc;                             // this context's last histogram (256 u64; hist[] may be all-reduced)
    const dc_dtable *plan_table;                  // the table and device total of the last plan
    uint64_t *plan_total;
    void *d_scr;            size_t scr_cap;       // per-wave garbage sinks of the decoders
    uint64_t *d_meta;                             // small device scalars
    uint4 *d_summ;          size_t summ_cap;
    uint64_t *d_entry;      size_t entry_cap;
    MtfSum *d_mtf;          size_t mtf_cap;       // adaptive nybble: tile summaries + entries, all levels
    uint8_t *d_rk;          size_t rk_cap;        // adaptive nybble: rank per element
    uint4 *d_mrec;          size_t mrec_cap;      // adaptive nybble: step records, MTF_REC per tile
    uint2 *d_mhead;         size_t mhead_cap;     // adaptive nybble: records per tile
    uint4 *d_fraw;          size_t fraw_cap;      // adaptive nybble: the encoder's tile summaries (k_mtf_resolve)
    bool summ_fresh;                              // d_summ holds them too (no scan since)
    MtfSum *h_mtf;                                // adaptive nybble: pinned entry lists (mtf_run)
    uint32_t *d_actl;       size_t actl_cap;      // adaptive nybble decode: control words of a segment
    uint32_t *d_astate;                           // adaptive nybble decode: lists + byte between segments
    const uint8_t *rk_in; uint64_t rk_len;        // identity of the input the ranks belong to
    const uint8_t *fsm_in; uint64_t fsm_len, fsm_nelem; int fsm_mode;   // input of the last transducer plan
    uint8_t *d_kscr;        size_t kscr_cap;      // chunked nybble: per-chunk streams before packing
    uint64_t *d_klens;      size_t klens_cap;     // chunked nybble: stream length per chunk
    uint64_t *h_pinned;                           // pinned host scalars
    const uint8_t *hist_in; uint64_t hist_n;      // identity of the last dc_huff_hist input
    bool hist_fe;                                 // ... histogram of its C5 front-end output (dc_small_huff_plan)
    bool plan_ok;
    // tuning options (dc_ctx_set_option; initial values from the environment, read once here)
    uint32_t opt_hist_grid;       // histogram workgroups (0: default 512)
    uint32_t opt_pack_grid;       // pack: workgroups of k_huff_pack (0: a block pair each; A/B builds: blocks per wave of k_huff_pack_w)
    uint32_t opt_pack_block;      // 2/3: the wave-per-range pack (k_huff_pack_w; 3: 4 codes a lane), A/B
    uint32_t opt_nyb_wtile_off;   // 1: the nybble encode / decode write with k_fsm_write (A/B, parity tests)
    uint32_t opt_d8_static;       // decoder: static share of the tuples, percent (0..100)
    uint32_t opt_decode_general;  // 1: always the general decoder (k_huff_decode)
    uint32_t opt_hist_pf;         // histogram: blocks of loads in flight ahead (1..2, 0 = default 2)
    uint32_t *d_hflag;            // histogram accumulator (256 u64) + done counter, zero between launches
    uint32_t opt_decode_variant;  // fast decoder: 0 one code per lookup (k_huff_decode8), 1 up to 3 (k_huff_decode9)
    uint32_t opt_adec_v1;         // adaptive nybble decode: 0 control words + k_nyb_resolve_c, 1 = the one-pass
                                  // k_nyb_adec, 2 = r2's k_nyb_resolve, 3 = k_nyb_resolve_s (A/B)
    // timing
    int timing;
    int nev;
    hipEvent_t ev0[DC_MAX_EVENTS], ev1[DC_MAX_EVENTS];
    const char *evname[DC_MAX_EVENTS];
    bool events_made;
};

#define HIPCHK(x) do { if ((x) != hipSuccess) return DC_E_HIP; } while (0)

// Decoder-table freshness. A pack builds the decoder tables of its table (its workgroup 0),
// so the decode after it skips k_dec_tables. The skip is keyed on the table's address AND on
// a process-wide generation that every table write through this library bumps (any context:
// k_huff_table, the fused encode plan): a table rebuilt since at the same address, e.g. a
// recycled buffer filled by another context, is never taken for the packed one. (Keyed on the
// address alone, such a table skipped the rebuild and its decode reported a stream error.)
static std::atomic<uint64_t> g_table_gen{1};
static void table_written(dc_ctx *c)
{
    c->dec_fresh = nullptr;
    g_table_gen.fetch_add(1, std::memory_order_relaxed);
}
static void dec_tables_built(dc_ctx *c, const dc_dtable *t)
{
    c->dec_fresh = t;
    c->dec_fresh_gen = g_table_gen.load(std::memory_order_relaxed);
}
static bool dec_tables_fresh(const dc_ctx *c, const dc_dtable *t)
{
    return c->dec_fresh == t && c->dec_fresh_gen == g_table_gen.load(std::memory_order_relaxed);
}

static int ensure(void **p, size_t *cap, size_t bytes)
{
    if (*cap >= bytes && *p) return DC_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    size_t want = bytes < 4096 ? 4096 : bytes;
    if (hipMalloc(p, want) != hipSuccess) { *p = nullptr; return DC_E_HIP; }
    *cap = want;
    return DC_OK;
}

static void t_begin(dc_ctx *c, const char *name, int *slot)
{
    *slot = -1;
    if (!c->timing || c->nev >= DC_MAX_EVENTS) return;
    *slot = c->nev++;
    c->evname[*slot] = name;
    (void)hipEventRecord(c->ev0[*slot], c->stream);
}
static void t_end(dc_ctx *c, int slot)
{
    if (slot >= 0) (void)hipEventRecord(c->ev1[slot], c->stream);
}

#define LAUNCH(ctx, name, kern, grid, block, ...) do {                         \
        int _slot; t_begin(ctx, name, &_slot);                                  \
        hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, ctx->stream, __VA_ARGS__); \
        if (hipGetLastError() != hipSuccess) return DC_E_HIP;                   \
        t_end(ctx, _slot);                                                      \
    } while (0)

static int g_rank_uploaded = -1;

extern "C" {

const char *dc_version(void) { return DC_VERSION; }
size_t dc_dtable_size(void) { return sizeof(dc_dtable); }

static int ctx_create(dc_ctx **out, int device, void *stream, bool own);

int dc_ctx_create(dc_ctx **out, int device, void *stream) { return ctx_create(out, device, stream, false); }
int dc_ctx_create_owned(dc_ctx **out, int device) { return ctx_create(out, device, nullptr, true); }

static int ctx_create(dc_ctx **out, int device, void *stream, bool own)
{
    if (!out) return DC_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device >= ndev) return DC_E_HIP;
    HIPCHK(hipSetDevice(device));
    dc_ctx *c = (dc_ctx *)calloc(1, sizeof(dc_ctx));
    if (!c) return DC_E_ARG;
    c->device = device;
    if (!own) { c->stream = (hipStream_t)stream; c->own_stream = false; }   // NULL = default stream
    else {
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { free(c); return DC_E_HIP; }
        c->own_stream = true;
    }
    if (hipMalloc((void **)&c->d_err, 16 * sizeof(int)) != hipSuccess ||
        hipMalloc((void **)&c->d_errp, 2 * 128 * sizeof(int)) != hipSuccess ||
        hipMemset(c->d_errp, 0, 2 * 128 * sizeof(int)) != hipSuccess ||
        hipMalloc((void **)&c->d_meta, 16 * sizeof(uint64_t)) != hipSuccess ||
        hipHostMalloc((void **)&c->h_pinned, 16 * sizeof(uint64_t), 0) != hipSuccess) {
        free(c);
        return DC_E_HIP;
    }
    c->d_errd = c->d_errp + 128;
    if (hipMalloc((void **)&c->d_hflag, 4096) != hipSuccess || hipMemset(c->d_hflag, 0, 4096) != hipSuccess ||
        hipMalloc((void **)&c->d_hloc, 256 * sizeof(uint64_t)) != hipSuccess ||
        hipMemset(c->d_hloc, 0, 256 * sizeof(uint64_t)) != hipSuccess) {
        free(c);
        return DC_E_HIP;
    }
    if (hipMalloc((void **)&c->d_queue, D8_QWORDS * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(c->d_queue, 0, D8_QWORDS * sizeof(uint32_t)) != hipSuccess) {
        free(c);
        return DC_E_HIP;
    }
    c->opt_d8_static = D8_STATIC_PCT;
    {   // A/B knobs (environment; tools/kern_ab.py sets the same options per context), read once and clamped
        const char *e;
        if ((e = getenv("DC_HIST_GRID"))) (void)dc_ctx_set_option(c, DC_OPT_HIST_GRID, atoll(e));
        if ((e = getenv("DC_PACK_GRID"))) (void)dc_ctx_set_option(c, DC_OPT_PACK_GRID, atoll(e));
        if ((e = getenv("DC_D8_STATIC"))) (void)dc_ctx_set_option(c, DC_OPT_DECODE_STATIC_PCT, atoll(e));
        if ((e = getenv("DC_DECODE_V7"))) (void)dc_ctx_set_option(c, DC_OPT_DECODE_GENERAL, atoll(e) != 0);
    }
    if (g_rank_uploaded != device) {
        uint8_t rank[256];
        memset(rank, 0xFF, sizeof(rank));
        const char *t = " etaoins";
        for (int r = 0; r < 8; ++r) rank[(uint8_t)t[r]] = (uint8_t)r;
        if (hipMemcpyToSymbol(HIP_SYMBOL(c_static_rank), rank, 256) != hipSuccess) { free(c); return DC_E_HIP; }
        g_rank_uploaded = device;
    }
    *out = c;
    return DC_OK;
}

void dc_ctx_destroy(dc_ctx *c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->d_bh) (void)hipFree(c->d_bh);
    if (c->d_off) (void)hipFree(c->d_off);
    if (c->d_plan) (void)hipFree(c->d_plan);
    if (c->d_msym) (void)hipFree(c->d_msym);
    if (c->d_gexp) (void)hipFree(c->d_gexp);
    if (c->d_err) (void)hipFree(c->d_err);
    if (c->d_errp) (void)hipFree(c->d_errp);
    if (c->d_hflag) (void)hipFree(c->d_hflag);
    if (c->d_hloc) (void)hipFree(c->d_hloc);
    if (c->d_queue) (void)hipFree(c->d_queue);
    if (c->d_fix) (void)hipFree(c->d_fix);
    if (c->d_fixpos) (void)hipFree(c->d_fixpos);
    if (c->d_scr) (void)hipFree(c->d_scr);
    if (c->d_meta) (void)hipFree(c->d_meta);
    if (c->d_summ) (void)hipFree(c->d_summ);
    if (c->d_entry) (void)hipFree(c->d_entry);
    if (c->d_mtf) (void)hipFree(c->d_mtf);
    if (c->d_rk) (void)hipFree(c->d_rk);
    if (c->d_mrec) (void)hipFree(c->d_mrec);
    if (c->d_mhead) (void)hipFree(c->d_mhead);
    if (c->d_fraw) (void)hipFree(c->d_fraw);
    if (c->h_mtf) (void)hipHostFree(c->h_mtf);
    if (c->d_actl) (void)hipFree(c->d_actl);
    if (c->d_astate) (void)hipFree(c->d_astate);
    if (c->d_kscr) (void)hipFree(c->d_kscr);
    if (c->d_klens) (void)hipFree(c->d_klens);
    if (c->h_pinned) (void)hipHostFree(c->h_pinned);
    if (c->events_made)
        for (int i = 0; i < DC_MAX_EVENTS; ++i) { (void)hipEventDestroy(c->ev0[i]); (void)hipEventDestroy(c->ev1[i]); }
    if (c->own_stream) (void)hipStreamDestroy(c->stream);
    free(c);
}

int dc_ctx_set_option(dc_ctx *c, int option, int64_t value)
{
    if (!c) return DC_E_ARG;
    switch (option) {
    case DC_OPT_HIST_GRID:   // 0 = default; the kernel's per-workgroup bin totals are u64
        if (value < 0 || value > (1 << 20)) return DC_E_ARG;
        c->opt_hist_grid = (uint32_t)value;
        return DC_OK;
    case DC_OPT_PACK_GRID:
        if (value < 0 || value > (1 << 24)) return DC_E_ARG;
        c->opt_pack_grid = (uint32_t)value;
        return DC_OK;
    case DC_OPT_DECODE_STATIC_PCT:
        if (value < 0 || value > 100) return DC_E_ARG;
        c->opt_d8_static = (uint32_t)value;
        return DC_OK;
    case DC_OPT_DECODE_GENERAL:
        if (value != 0 && value != 1) return DC_E_ARG;
        c->opt_decode_general = (uint32_t)value;
        return DC_OK;
    case DC_OPT_DECODE_VARIANT:   // 1: k_huff_decode9, in DC_AB_KERNELS builds only
#ifdef DC_AB_KERNELS
        if (value < 0 || value > 1) return DC_E_ARG;
#else
        if (value != 0) return DC_E_ARG;
#endif
        c->opt_decode_variant = (uint32_t)value;
        return DC_OK;
    case DC_OPT_NYB_ADEC_V1:   // 1-3: the A/B resolves, in DC_AB_KERNELS builds only
#ifdef DC_AB_KERNELS
        if (value < 0 || value > 3) return DC_E_ARG;
#else
        if (value != 0) return DC_E_ARG;
#endif
        c->opt_adec_v1 = (uint32_t)value;
        return DC_OK;
    case DC_OPT_HIST_PREFETCH:
        if (value < 0 || value > 3) return DC_E_ARG;
        c->opt_hist_pf = (uint32_t)value;
        return DC_OK;
    case DC_OPT_PACK_BLOCK:   // 2/3: k_huff_pack_w, in DC_AB_KERNELS builds only
#ifdef DC_AB_KERNELS
        if (value < 0 || value > 7) return DC_E_ARG;
#else
        if (value != 0) return DC_E_ARG;
#endif
        c->opt_pack_block = (uint32_t)value;
        return DC_OK;
    case DC_OPT_NYB_WTILE_OFF:
        if (value != 0 && value != 1) return DC_E_ARG;
        c->opt_nyb_wtile_off = (uint32_t)value;
        return DC_OK;
    default:
        return DC_E_ARG;
    }
}

int dc_ctx_sync(dc_ctx *c) { return (c && hipStreamSynchronize(c->stream) == hipSuccess) ? DC_OK : DC_E_HIP; }
void *dc_ctx_stream(dc_ctx *c) { return c ? (void *)c->stream : nullptr; }

int dc_ctx_set_timing(dc_ctx *c, int enable)
{
    if (!c) return DC_E_ARG;
    if (enable && !c->events_made) {
        for (int i = 0; i < DC_MAX_EVENTS; ++i) {
            HIPCHK(hipEventCreate(&c->ev0[i]));
            HIPCHK(hipEventCreate(&c->ev1[i]));
        }
        c->events_made = true;
    }
    c->timing = enable;
    c->nev = 0;
    return DC_OK;
}

int dc_ctx_timings(dc_ctx *c, const char **names, float *ms, int max)
{
    if (!c) return DC_E_ARG;
    HIPCHK(hipStreamSynchronize(c->stream));
    int n = c->nev < max ? c->nev : max;
    for (int i = 0; i < n; ++i) {
        names[i] = c->evname[i];
        float v = 0.f;
        HIPCHK(hipEventElapsedTime(&v, c->ev0[i], c->ev1[i]));
        ms[i] = v;
    }
    return n;
}

int dc_malloc(void **p, size_t bytes) { return hipMalloc(p, bytes ? bytes : 1) == hipSuccess ? DC_OK : DC_E_HIP; }
int dc_free(void *p) { return hipFree(p) == hipSuccess ? DC_OK : DC_E_HIP; }
int dc_memcpy_h2d(dc_ctx *c, void *d, const void *h, size_t bytes)
{
    if (!bytes) return DC_OK;
    HIPCHK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return DC_OK;
}
int dc_memcpy_d2h(dc_ctx *c, void *h, const void *d, size_t bytes)
{
    if (!bytes) return DC_OK;
    HIPCHK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return DC_OK;
}
int dc_memset(dc_ctx *c, void *d, int v, size_t bytes)
{
    if (!bytes) return DC_OK;
    HIPCHK(hipMemsetAsync(d, v, bytes, c->stream));
    return DC_OK;
}
int dc_copy_probe(dc_ctx *c, const void *d_src, void *d_dst, uint64_t bytes)
{
    if (!c || (bytes && (!d_src || !d_dst)) || (bytes & 15) || (((uintptr_t)d_src | (uintptr_t)d_dst) & 15)) return DC_E_ARG;
    if (!bytes) return DC_OK;
    // the full grid, one uint4 per lane (6.34 TB/s on 1 GiB, k_copy_probe's comment); grid-
    // stride beyond 2^31 - 1 workgroups (32 TiB)
    const uint64_t n16 = bytes / 16, wgs = (n16 + 255) / 256;
    LAUNCH(c, "copy_probe", k_copy_probe, wgs < 0x7fffffffull ? wgs : 0x7fffffffull, 256, (const uint4 *)d_src,
           (uint4 *)d_dst, n16);
    return DC_OK;
}

// ---- Huffman -----------------------------------------------------------------------
static uint64_t nblocks_of(uint64_t n) { return (n + DC_BLOCK_BYTES - 1) / DC_BLOCK_BYTES; }

static int hist_impl(dc_ctx *c, const uint8_t *d_in, uint64_t n, uint64_t *d_hist, HistFuse fuse, bool fe = false,
                     const int64_t *shard = nullptr)
{
    if (!c || !d_hist || (n && !d_in)) return DC_E_ARG;
    if (((uintptr_t)d_in) & 15) return DC_E_ARG;
    const uint64_t nb = nblocks_of(n);
    if (ensure((void **)&c->d_bh, &c->bh_cap, (nb ? nb : 1) * 256 * sizeof(uint16_t))) return DC_E_HIP;
    c->hist_in = d_in;
    c->hist_n = n;
    c->hist_fe = fe;
    c->plan_ok = false;
    if (fe) {   // n >= 2 (dc_small_huff_plan)
        const uint64_t grid = nb < 512u ? nb : 512u;
        LAUNCH(c, "fe_hist_blocks", (k_hist_blocks<1, true>), grid, 256, d_in, n, nb, c->d_bh, d_hist,
               reinterpret_cast<uint64_t *>(c->d_hflag), c->d_hflag + 512, c->d_hloc, fuse, shard);
        return DC_OK;
    }
    if (nb == 0) {
        HIPCHK(hipMemsetAsync(d_hist, 0, 256 * sizeof(uint64_t), c->stream));
        HIPCHK(hipMemsetAsync(c->d_hloc, 0, 256 * sizeof(uint64_t), c->stream));
        if (fuse.T) LAUNCH(c, "huff_table", k_huff_table, 1, 256, (const uint64_t *)c->d_hloc, 1, (const int32_t *)nullptr,
                           fuse.M, fuse.nary, fuse.T, (dc_tree *)nullptr, (const uint64_t *)c->d_hloc, fuse.d_total,
                           fuse.perr, fuse.perr_next);
        return DC_OK;
    }
    const uint64_t hmax = c->opt_hist_grid ? c->opt_hist_grid : 512u;
    const uint64_t grid = nb < hmax ? nb : hmax;   // 512: 2 resident per CU (64 KiB LDS each)
    // two blocks of loads in flight ahead (with nt loads; same-box A/B in the 1 GiB C2 step:
    // 0.176 ms against 0.179 with one; before the nt loads one was best, 0.1995 vs 0.2022 ms)
    uint64_t *const hacc = reinterpret_cast<uint64_t *>(c->d_hflag);
    uint32_t *const hdone = c->d_hflag + 512;
    if (c->opt_hist_pf == 1)
        LAUNCH(c, "hist_blocks", k_hist_blocks<1>, grid, 256, d_in, n, nb, c->d_bh, d_hist, hacc, hdone, c->d_hloc, fuse);
    else if (c->opt_hist_pf == 3)
        LAUNCH(c, "hist_blocks", k_hist_blocks<3>, grid, 256, d_in, n, nb, c->d_bh, d_hist, hacc, hdone, c->d_hloc, fuse);
    else LAUNCH(c, "hist_blocks", k_hist_blocks<2>, grid, 256, d_in, n, nb, c->d_bh, d_hist, hacc, hdone, c->d_hloc, fuse);
    return DC_OK;
}

int dc_huff_hist(dc_ctx *c, const uint8_t *d_in, uint64_t n, uint64_t *d_hist)
{
    return hist_impl(c, d_in, n, d_hist, HistFuse{nullptr, 0, 0, nullptr, nullptr, nullptr});
}

static int table_common(dc_ctx *c, const uint64_t *d_freq, int is_hist, const int32_t *d_len, int M,
                        int nary, dc_dtable *d_table)
{
    if (!c || !d_table || M < 0 || M >= DC_MAX_SYMS || nary < 2 || nary > 256) return DC_E_ARG;
    table_written(c);
    LAUNCH(c, "huff_table", k_huff_table, 1, 256, d_freq, is_hist, d_len, M, nary, d_table, (dc_tree *)nullptr,
           (const uint64_t *)nullptr, (uint64_t *)nullptr, (int *)nullptr, (int *)nullptr);
    return DC_OK;
}

int dc_huff_tree(dc_ctx *c, const uint64_t *d_freq, int M, int nary, dc_dtable *d_table, dc_tree *d_tree)
{
    if (!c || !d_freq || !d_table || !d_tree || M < 0 || M >= DC_MAX_SYMS || nary < 2 || nary > 256) return DC_E_ARG;
    table_written(c);
    LAUNCH(c, "huff_tree", k_huff_table, 1, 256, d_freq, 0, (const int32_t *)nullptr, M, nary, d_table, d_tree,
           (const uint64_t *)nullptr, (uint64_t *)nullptr, (int *)nullptr, (int *)nullptr);
    return DC_OK;
}

int dc_tree_depths(dc_ctx *c, const int32_t *d_parent, int list_length, int leaves, int32_t *d_depth)
{
    if (!c || !d_parent || !d_depth || list_length < 1 || leaves < 0 || leaves > list_length) return DC_E_ARG;
    if (leaves == 0) return DC_OK;
    LAUNCH(c, "tree_depths", k_tree_depths, (leaves + 255) / 256, 256, d_parent, list_length, leaves, d_depth);
    return DC_OK;
}

int dc_huff_table(dc_ctx *c, const uint64_t *d_hist, int M, int nary, dc_dtable *d_table)
{
    if (!d_hist) return DC_E_ARG;
    return table_common(c, d_hist, 1, nullptr, M, nary, d_table);
}
int dc_huff_table_freq(dc_ctx *c, const uint64_t *d_freq, int M, int nary, dc_dtable *d_table)
{
    if (!d_freq) return DC_E_ARG;
    return table_common(c, d_freq, 0, nullptr, M, nary, d_table);
}
int dc_huff_table_lengths(dc_ctx *c, const int32_t *d_len, int M, int nary, dc_dtable *d_table)
{
    if (!d_len) return DC_E_ARG;
    return table_common(c, nullptr, 0, d_len, M, nary, d_table);
}

int dc_huff_table_status(dc_ctx *c, const dc_dtable *d_table, int32_t *max_bits)
{
    int32_t v[2];
    HIPCHK(hipMemcpyAsync(v, &d_table->max_bits, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(v + 1, &d_table->status, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (max_bits) *max_bits = v[0];
    return v[1];
}

static int *plan_err(dc_ctx *c) { return c->d_errp + 4 * (c->gen_p & 31u); }
static int *plan_err_next(dc_ctx *c) { return c->d_errp + 4 * ((c->gen_p + 1) & 31u); }
static int *dec_err(dc_ctx *c) { return c->d_errd + 4 * (c->gen_d & 31u); }
static int *dec_err_next(dc_ctx *c) { return c->d_errd + 4 * ((c->gen_d + 1) & 31u); }

int dc_huff_plan(dc_ctx *c, const dc_dtable *d_table, uint64_t *d_total_bits)
{
    if (!c || !d_table || !d_total_bits) return DC_E_ARG;
    if (!c->hist_in && c->hist_n) return DC_E_STATE;
    ++c->gen_p;   // this plan's error slot (cleared by the plan before; the next one is cleared below)
    // the payload bits of this context's last histogram under d_table (and the missing-code
    // flag): one 256-thread launch; the blocks' offsets come from the plan kernels the pack
    // launches first (plan_offsets: k_block_local + k_block_final_wide)
    LAUNCH(c, "plan_total", k_plan_total, 1, 256, (const uint64_t *)c->d_hloc, d_table, d_total_bits, plan_err(c),
           plan_err_next(c));
    c->plan_table = d_table;
    c->plan_total = d_total_bits;
    c->plan_ok = true;
    return DC_OK;
}

int dc_huff_table_plan(dc_ctx *c, const uint64_t *d_hist, int M, int nary, dc_dtable *d_table, uint64_t *d_total_bits)
{
    if (!c || !d_hist || !d_table || !d_total_bits || M < 0 || M >= DC_MAX_SYMS || nary < 2 || nary > 256) return DC_E_ARG;
    if (!c->hist_in && c->hist_n) return DC_E_STATE;
    ++c->gen_p;   // this plan's error slot (the table kernel clears the next one)
    table_written(c);
    // the table of d_hist (e.g. the all-reduced histogram of every shard) and, in the same
    // launch, the payload bits of THIS context's last histogram under it (huff_table_body's plan)
    LAUNCH(c, "huff_table", k_huff_table, 1, 256, d_hist, 1, (const int32_t *)nullptr, M, nary, d_table,
           (dc_tree *)nullptr, (const uint64_t *)c->d_hloc, d_total_bits, plan_err(c), plan_err_next(c));
    c->plan_table = d_table;
    c->plan_total = d_total_bits;
    c->plan_ok = true;
    return DC_OK;
}

int dc_huff_encode_plan(dc_ctx *c, const uint8_t *d_in, uint64_t n, int M, int nary, uint64_t *d_hist,
                        dc_dtable *d_table, uint64_t *d_total_bits)
{
    if (!c || !d_table || !d_total_bits || M < 0 || M >= DC_MAX_SYMS || nary < 2 || nary > 256) return DC_E_ARG;
    ++c->gen_p;
    table_written(c);
    const int r = hist_impl(c, d_in, n, d_hist,
                            HistFuse{d_table, M, nary, d_total_bits, plan_err(c), plan_err_next(c)});
    if (r != DC_OK) { --c->gen_p; return r; }
    c->plan_table = d_table;
    c->plan_total = d_total_bits;
    c->plan_ok = true;
    return DC_OK;
}

// The per-block exclusive bit offsets of the last histogram's input under c->plan_table into
// c->d_off (nblocks + 1 entries), and with d_words set the zeroed block-boundary words the
// pack OR-merges into: two launches (one more above PLAN_MAX_WG workgroups of blocks)
// With sl32 set (C5 fused front-end, k_fe_pack): also the symbol index of each block's first
// symbol into c->d_msym, and the sync-length dwords of the chunks spanning block boundaries
// zeroed (S = 1 << slog); one plan launch pair as well, at most PLAN_MAX_WG workgroups.
static int plan_offsets(dc_ctx *c, int *err, int *err_next, uint64_t bit_base, const uint64_t *d_base,
                        uint32_t *d_words, uint64_t words_cap, uint32_t *sl32 = nullptr, uint32_t slog = 0,
                        const int64_t *shard = nullptr, uint32_t *gl32 = nullptr)
{
    const uint64_t nb = nblocks_of(c->hist_n);
    if (ensure((void **)&c->d_off, &c->off_cap, (nb + 1) * sizeof(uint64_t))) return DC_E_HIP;
    if (nb == 0) {
        if (sl32) return DC_E_ARG;
        HIPCHK(hipMemsetAsync(c->d_off, 0, sizeof(uint64_t), c->stream));
        return DC_OK;
    }
    const uint64_t nwg = (nb + PLAN_WG_BLOCKS - 1) / PLAN_WG_BLOCKS;
    if (nwg <= PLAN_MAX_WG) {
        if (ensure((void **)&c->d_plan, &c->plan_cap, 2 * (nb + nwg + 64) * sizeof(uint32_t))) return DC_E_HIP;
        uint32_t *loc = c->d_plan, *tot = c->d_plan + nb + 32;
        uint32_t *lcnt = nullptr, *wgcnt = nullptr;
        if (sl32) {
            if (ensure((void **)&c->d_msym, &c->msym_cap, (nb + 1) * sizeof(uint64_t))) return DC_E_HIP;
            lcnt = c->d_plan + nb + nwg + 64;
            wgcnt = lcnt + nb + 32;
        }
        LAUNCH(c, "block_bits", k_block_local, nwg, 256, (const uint16_t *)c->d_bh, nb, c->plan_table, loc, tot, err,
               lcnt, wgcnt);
        LAUNCH(c, "block_scan", k_block_final_wide, nwg, 256, (const uint32_t *)loc, (const uint32_t *)tot, nb,
               (uint32_t)nwg, c->d_off, c->d_meta + 15, err_next, bit_base, d_base, d_words, words_cap,
               (const uint32_t *)lcnt, (const uint32_t *)wgcnt, c->d_msym, sl32, slog, shard, gl32);
    } else if (sl32) {
        return DC_E_ARG;
    } else {
        LAUNCH(c, "block_bits", k_block_bits, (nb + 3) / 4, 256, (const uint16_t *)c->d_bh, nb, c->plan_table,
               c->d_off, err);
        LAUNCH(c, "block_scan", k_block_scan, 1, 1024, c->d_off, nb, c->d_meta + 15, err_next);
        if (d_words)
            LAUNCH(c, "zero_bounds", k_zero_bounds, (nb + 1 + 255) / 256, 256, (const uint64_t *)c->d_off, nb, bit_base,
                   d_base, d_words, words_cap);
    }
    return DC_OK;
}

int dc_huff_plan_offsets(dc_ctx *c, uint64_t *h_off, uint64_t max_entries, uint64_t *h_n)
{
    // inspection (synchronising): the offsets of the last plan, recomputed by the plan kernels
    if (!c || !c->plan_ok || !c->plan_table) return DC_E_STATE;
    const uint64_t nb = nblocks_of(c->hist_n);
    if (h_n) *h_n = nb + 1;
    const uint64_t k = nb + 1 < max_entries ? nb + 1 : max_entries;
    int *const scratch_err = c->d_err + 12;   // not a plan slot: the flags of the real plan stay
    const int r = plan_offsets(c, scratch_err, scratch_err, 0, nullptr, nullptr, 0);
    if (r != DC_OK) return r;
    if (k) {
        HIPCHK(hipMemcpyAsync(h_off, c->d_off, k * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return DC_OK;
}

int dc_huff_block_hist(dc_ctx *c, uint16_t *h_bh, uint64_t max_entries)
{
    if (!c || !c->hist_n) return DC_E_STATE;
    const uint64_t nb = nblocks_of(c->hist_n) * 256;
    const uint64_t k = nb < max_entries ? nb : max_entries;
    HIPCHK(hipMemcpyAsync(h_bh, c->d_bh, k * sizeof(uint16_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return DC_OK;
}

uint64_t dc_huff_words_needed(uint64_t bit_base, uint64_t total_bits)
{
    return (((bit_base & 31) + total_bits + 31) >> 5) + 24;   // + slack: the decoder prefetches 64 B ahead
}

static bool sync_ok(uint32_t S) { return S >= 16 && S <= DC_SYNC_MAX && (S & (S - 1)) == 0; }

uint64_t dc_huff_sync_chunks(uint64_t n, uint32_t S) { return S ? (n + S - 1) / S : 0; }
uint64_t dc_huff_sync_groups(uint64_t n, uint32_t S) { return (dc_huff_sync_chunks(n, S) + DC_SYNC_GROUP - 1) / DC_SYNC_GROUP; }


static int pack_impl(dc_ctx *c, const uint8_t *d_in, uint64_t n, const dc_dtable *d_table, uint64_t bit_base,
                     const uint64_t *d_base, uint32_t *d_words, uint64_t words_cap, uint64_t *d_sync_base,
                     uint16_t *d_sync_len, uint32_t sync_syms)
{
    if (!c || !d_table || !d_words) return DC_E_ARG;
    if (d_in != c->hist_in || n != c->hist_n || c->hist_fe || !c->plan_ok || !c->plan_total) return DC_E_STATE;
    if ((d_sync_base != nullptr) != (d_sync_len != nullptr)) return DC_E_ARG;
    if (d_sync_len && !sync_ok(sync_syms)) return DC_E_ARG;
    const uint64_t nb = nblocks_of(n);
    if (nb == 0) return DC_OK;
    // the blocks' offsets, and the boundary words zeroed (the plan's error flags: its slot)
    const int r = plan_offsets(c, plan_err(c), plan_err_next(c), bit_base, d_base, d_words, words_cap);
    if (r != DC_OK) return r;
#ifdef DC_AB_KERNELS
    if (c->opt_pack_block == 7) {   // A/B: the next block's pieces loaded as pass B frees them, persistent grid
        int ncu = 256;
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device);
        const uint64_t gmax = c->opt_pack_grid ? c->opt_pack_grid : (uint64_t)ncu * 4;
        const uint64_t grid = nb < gmax ? nb : gmax;
        LAUNCH(c, "huff_pack", k_huff_pack<true>, grid + 1, 256, d_in, n, d_table, (const uint64_t *)c->d_off, bit_base,
               d_base, d_words, d_sync_base, d_sync_len, sync_syms, nb, words_cap, plan_err(c), 1);
    } else if (c->opt_pack_block == 6) {   // A/B: one code-table read per byte (k_huff_pack_fold)
        const uint64_t gmax = c->opt_pack_grid ? c->opt_pack_grid : (nb + 1) / 2;
        const uint64_t grid = nb < gmax ? nb : gmax;
        LAUNCH(c, "huff_pack", k_huff_pack_fold, grid + 1, 256, d_in, n, d_table, (const uint64_t *)c->d_off, bit_base,
               d_base, d_words, d_sync_base, d_sync_len, sync_syms, nb, words_cap, plan_err(c), 1);
    } else if (c->opt_pack_block == 5) {   // A/B: a half-block stage, more workgroups per CU (k_huff_pack_half)
        LAUNCH(c, "huff_pack", k_huff_pack_half, (nb + 1) / 2, 256, d_in, n, d_table, (const uint64_t *)c->d_off,
               bit_base, d_base, d_words, d_sync_base, d_sync_len, sync_syms, nb, words_cap, plan_err(c));
    } else if (c->opt_pack_block == 4) {   // A/B: the next block in flight by LDS-DMA (k_huff_pack_dma)
        int ncu = 256;
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device);
        const uint64_t grid = (uint64_t)ncu * PKD_WG_PER_CU;
        LAUNCH(c, "huff_pack", k_huff_pack_dma, (nb < grid ? nb : grid) + 1, 256, d_in, n, d_table,
               (const uint64_t *)c->d_off, bit_base, d_base, d_words, d_sync_base, d_sync_len, sync_syms, nb, words_cap,
               plan_err(c), 1);
    } else if ((((uintptr_t)d_words) & 15) == 0 && c->opt_pack_block >= 2 && n >= 1024) {   // A/B: 0.386 vs 0.380 ms
        if (ensure((void **)&c->d_scr, &c->scr_cap, (size_t)D8_SCRATCH_WAVES * D8_WSCR)) return DC_E_HIP;   // trash rows
        // one wave per range of bpw blocks (k_huff_pack_w): ~PW_WAVES waves, 4 per workgroup,
        // + workgroup 0: the decoder tables (k_huff_table leaves them to the pack's idle CU time)
        const uint64_t bpw = c->opt_pack_grid ? c->opt_pack_grid : (nb + PW_WAVES - 1) / PW_WAVES;
        const uint64_t waves = (nb + bpw - 1) / bpw;
        LAUNCH(c, "huff_pack", k_huff_pack_w, (waves + 3) / 4 + 1, 256, d_in, n, d_table, (const uint64_t *)c->d_off,
               bit_base, d_base, d_words, d_sync_base, d_sync_len, sync_syms, nb, words_cap, plan_err(c), 1,
               (uint32_t)bpw, (uint8_t *)c->d_scr, c->opt_pack_block == 3 ? 1 : 0);
    } else
#endif
    {
        // two blocks per workgroup (grid-stride) + workgroup 0: the decoder tables
        const uint64_t gmax = c->opt_pack_grid ? c->opt_pack_grid : (nb + 1) / 2;
        const uint64_t grid = nb < gmax ? nb : gmax;
        LAUNCH(c, "huff_pack", k_huff_pack<>, grid + 1, 256, d_in, n, d_table, (const uint64_t *)c->d_off, bit_base,
               d_base, d_words, d_sync_base, d_sync_len, sync_syms, nb, words_cap, plan_err(c), 1);
    }
    dec_tables_built(c, d_table);   // workgroup 0 built the decoder tables
    return DC_OK;
}

int dc_huff_pack_async(dc_ctx *c, const uint8_t *d_in, uint64_t n, const dc_dtable *d_table, uint64_t bit_base,
                       uint32_t *d_words, uint64_t words_cap, uint64_t *d_sync_base, uint16_t *d_sync_len,
                       uint32_t sync_syms)
{
    return pack_impl(c, d_in, n, d_table, bit_base, nullptr, d_words, words_cap, d_sync_base, d_sync_len, sync_syms);
}

int dc_huff_pack_async_dev(dc_ctx *c, const uint8_t *d_in, uint64_t n, const dc_dtable *d_table,
                           const uint64_t *d_bit_base, uint32_t *d_words, uint64_t words_cap, uint64_t *d_sync_base,
                           uint16_t *d_sync_len, uint32_t sync_syms)
{
    if (!d_bit_base) return DC_E_ARG;
    return pack_impl(c, d_in, n, d_table, 0, d_bit_base, d_words, words_cap, d_sync_base, d_sync_len, sync_syms);
}

// ---- C5 fused front-end encode (k_hist_blocks<.., true> + plan + k_fe_pack) -------------
int dc_small_huff_plan(dc_ctx *c, const uint8_t *d_in, uint64_t n, int M, int nary, uint64_t *d_hist,
                       dc_dtable *d_table, uint64_t *d_total_bits)
{
    if (!c || !d_table || !d_total_bits || !d_hist || M < 255 || M >= DC_MAX_SYMS || nary < 2 || nary > 256) return DC_E_ARG;
    if (n < 2) return DC_E_FALLBACK;   // the front-end output of < 2 bytes is LITERAL
    ++c->gen_p;
    table_written(c);
    const int r = hist_impl(c, d_in, n, d_hist, HistFuse{d_table, M, nary, d_total_bits, plan_err(c), plan_err_next(c)},
                            true);
    if (r != DC_OK) { --c->gen_p; return r; }
    c->plan_table = d_table;
    c->plan_total = d_total_bits;
    c->plan_ok = true;
    return DC_OK;
}

int dc_small_huff_pack_async(dc_ctx *c, const uint8_t *d_in, uint64_t n, const dc_dtable *d_table, uint64_t bit_base,
                             uint32_t *d_words, uint64_t words_cap, uint64_t *d_sync_base, uint16_t *d_sync_len,
                             uint32_t sync_syms)
{
    if (!c || !d_table || !d_words || !d_sync_base || !d_sync_len || !sync_ok(sync_syms)) return DC_E_ARG;
    if (((uintptr_t)d_sync_len) & 3) return DC_E_ARG;
    if (d_in != c->hist_in || n != c->hist_n || !c->hist_fe || !c->plan_ok || !c->plan_total) return DC_E_STATE;
    const uint64_t nb = nblocks_of(n);
    const int r = plan_offsets(c, plan_err(c), plan_err_next(c), bit_base, nullptr, d_words, words_cap,
                               reinterpret_cast<uint32_t *>(d_sync_len), (uint32_t)__builtin_ctz(sync_syms));
    if (r != DC_OK) return r;
    const uint64_t gmax = c->opt_pack_grid ? c->opt_pack_grid : (nb + 1) / 2;
    const uint64_t grid = nb < gmax ? nb : gmax;
    LAUNCH(c, "fe_pack", k_fe_pack<false>, grid + 1, 256, d_in, n, d_table, (const uint64_t *)c->d_off,
           (const uint64_t *)c->d_msym, bit_base, d_words, d_sync_base, d_sync_len, sync_syms, nb, words_cap,
           plan_err(c), 1, (const int64_t *)nullptr, (uint64_t *)nullptr, (uint16_t *)nullptr);
    dec_tables_built(c, d_table);
    return DC_OK;
}

// ---- C5 fused front-end encode of a shard (dist.ShardedSmall at world > 1) ---------------
// The shard's front-end histogram (the bytes either side from d_shard: FeShard), no table: the
// caller all-reduces the histograms, then dc_huff_table_plan builds the stream's table and this
// shard's payload bits under it.
int dc_small_huff_shard_hist(dc_ctx *c, const uint8_t *d_in, uint64_t n, const int64_t *d_shard, uint64_t *d_hist)
{
    if (!c || !d_shard || !d_hist) return DC_E_ARG;
    if (n < 2) return DC_E_FALLBACK;
    return hist_impl(c, d_in, n, d_hist, HistFuse{nullptr, 0, 0, nullptr, nullptr, nullptr}, true, d_shard);
}

// The shard's codes at the global bit d_shard[0] (d_words: word 0 = global word d_shard[0] / 32),
// its local sync index (its own decode) and its part of the stream's global sync index
// (k_fe_pack<true>). Nothing is read back: the offsets stay on the device.
int dc_small_huff_shard_pack_async(dc_ctx *c, const uint8_t *d_in, uint64_t n, const dc_dtable *d_table,
                                   const int64_t *d_shard, uint32_t *d_words, uint64_t words_cap,
                                   uint64_t *d_sync_base, uint16_t *d_sync_len, uint64_t *d_gsync_base,
                                   uint16_t *d_gsync_len, uint32_t sync_syms)
{
    if (!c || !d_table || !d_shard || !d_words || !d_sync_base || !d_sync_len || !d_gsync_base || !d_gsync_len ||
        !sync_ok(sync_syms))
        return DC_E_ARG;
    if ((((uintptr_t)d_sync_len) & 3) || (((uintptr_t)d_gsync_len) & 3)) return DC_E_ARG;
    if (d_in != c->hist_in || n != c->hist_n || !c->hist_fe || !c->plan_ok || !c->plan_total) return DC_E_STATE;
    const uint64_t nb = nblocks_of(n);
    const uint32_t slog = (uint32_t)__builtin_ctz(sync_syms);
    const int r = plan_offsets(c, plan_err(c), plan_err_next(c), 0, reinterpret_cast<const uint64_t *>(d_shard),
                               d_words, words_cap, reinterpret_cast<uint32_t *>(d_sync_len), slog, d_shard,
                               reinterpret_cast<uint32_t *>(d_gsync_len));
    if (r != DC_OK) return r;
    const uint64_t gmax = c->opt_pack_grid ? c->opt_pack_grid : (nb + 1) / 2;
    const uint64_t grid = nb < gmax ? nb : gmax;
    LAUNCH(c, "fe_pack", k_fe_pack<true>, grid + 1, 256, d_in, n, d_table, (const uint64_t *)c->d_off,
           (const uint64_t *)c->d_msym, (uint64_t)0, d_words, d_sync_base, d_sync_len, sync_syms, nb, words_cap,
           plan_err(c), 1, d_shard, d_gsync_base, d_gsync_len);
    dec_tables_built(c, d_table);
    return DC_OK;
}

int dc_small_huff_symbols(dc_ctx *c, uint64_t *h_m)
{
    if (!c || !h_m) return DC_E_ARG;
    if (!c->hist_fe || !c->d_msym || !c->hist_n) return DC_E_STATE;
    HIPCHK(hipMemcpyAsync(h_m, c->d_msym + nblocks_of(c->hist_n), sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return DC_OK;
}

uint32_t dc_huff_plan_gen(dc_ctx *c) { return c ? c->gen_p : 0u; }

int dc_huff_pack_status(dc_ctx *c, const dc_dtable *d_table)
{
    if (!c) return DC_E_ARG;
    return dc_huff_pack_status_gen(c, d_table, c->gen_p);
}

int dc_huff_pack_status_gen(dc_ctx *c, const dc_dtable *d_table, uint32_t gen)
{
    if (!c) return DC_E_ARG;
    // the plan's own slot; 32 slots rotate, and plan gen + 1's slot is cleared by plan gen:
    // a plan more than 30 plans back has lost its flags
    if ((uint32_t)(c->gen_p - gen) > 30u) return DC_E_STATE;
    int v[3] = {0, 0, 0};
    HIPCHK(hipMemcpyAsync(v, c->d_errp + 4 * (gen & 31u), 3 * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (v[0]) {
        const int st = dc_huff_table_status(c, d_table, nullptr);
        return st ? st : DC_E_NOCODE;
    }
    if (v[1]) return DC_E_FALLBACK;   // k_fe_pack: the fused path does not apply
    return v[2] ? DC_E_CAPACITY : DC_OK;
}

int dc_huff_pack(dc_ctx *c, const uint8_t *d_in, uint64_t n, const dc_dtable *d_table, uint64_t bit_base,
                 uint32_t *d_words, uint64_t words_cap, uint64_t *d_sync_base, uint16_t *d_sync_len,
                 uint32_t sync_syms)
{
    if (!c || !d_table || !d_words) return DC_E_ARG;
    if (d_in != c->hist_in || n != c->hist_n || !c->plan_ok || !c->plan_total) return DC_E_STATE;
    if ((d_sync_base != nullptr) != (d_sync_len != nullptr)) return DC_E_ARG;
    if (d_sync_len && !sync_ok(sync_syms)) return DC_E_ARG;
    // plan errors (a byte without a code) are checked here: host read of one int
    int err = 0;
    HIPCHK(hipMemcpyAsync(c->h_pinned, plan_err(c), sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(c->h_pinned + 1, c->plan_total, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    err = *(int *)c->h_pinned;
    if (err) {
        const int st = dc_huff_table_status(c, d_table, nullptr);
        return st ? st : DC_E_NOCODE;
    }
    const uint64_t total = c->h_pinned[1];
    if (dc_huff_words_needed(bit_base, total) > words_cap) return DC_E_CAPACITY;
    return dc_huff_pack_async(c, d_in, n, d_table, bit_base, d_words, words_cap, d_sync_base, d_sync_len, sync_syms);
}

uint32_t dc_huff_default_sync(uint64_t n)
{
    (void)n;
    return 64;
}

uint32_t dc_huff_choose_sync(uint64_t n, uint64_t total_bits)
{
    // 64 symbols per chunk: the decoder stages a group's input (4.5 KiB) and output (64 x
    // 64 B) through LDS. Denser streams (> ~8.5 bits/symbol) use 32 so the input still fits.
    if (n == 0) return 64;
    const double avg = (double)total_bits / (double)n;
    return (64.0 * 64.0 * avg / 8.0 <= 4200.0) ? 64u : 32u;
}

// d_gexp (C5, dc_small_huff_decode): symbols >= 0x80 per group of 64 chunks, from the fast
// decoder and its redo (S = 64 only: DC_E_ARG otherwise)
static int decode_impl(dc_ctx *c, const uint32_t *d_words, uint64_t bit_base, const uint64_t *d_base, uint64_t words,
                       const uint64_t *d_sync_base, const uint16_t *d_sync_len, uint32_t S, uint64_t n,
                       const dc_dtable *d_table, uint8_t *d_out, uint32_t *d_gexp = nullptr)
{
    if (!c || !d_table || (n && (!d_words || !d_sync_base || !d_sync_len || !d_out))) return DC_E_ARG;
    if (!sync_ok(S)) return DC_E_ARG;
    if (((uintptr_t)d_out) & 15) return DC_E_ARG;
    if (((uintptr_t)d_words) & 15) return DC_E_ARG;
    if (n == 0) return DC_OK;
    if (words < 4) return DC_E_ARG;
    const uint64_t groups = dc_huff_sync_groups(n, S);
    ++c->gen_d;   // this decode's error slot (cleared by the decode before; it clears the next one)
    int *const derr = dec_err(c), *const derr_next = dec_err_next(c);
    // the decoder tables, unless this context's last pack built them for this table (no launch
    // then; a table rebuilt elsewhere since reads dec_ready 0 in the decoder: a stream error)
    if (!dec_tables_fresh(c, d_table)) LAUNCH(c, "dec_tables", k_dec_tables, 1, 256, const_cast<dc_dtable *>(d_table), derr);
    const bool fast8 = S == 64 && n < (1ull << 37) && words < (1ull << 31) && !c->opt_decode_general;
    if (d_gexp && (!fast8 || c->opt_decode_variant != 0)) return DC_E_ARG;   // (k_huff_decode9 writes no counts)
    if (fast8) {
        // 12 waves x 2 chains, one workgroup per CU: the stage and the 14-bit table fill the
        // LDS (the 8 x 4 split measured 0.89 vs 0.70 ms on 1 GiB C2: spills)
        const uint32_t spct = c->opt_d8_static;   // clamped to 0..100 by dc_ctx_set_option
        const uint64_t tuples = (groups + 1) / 2;   // 2 chains (groups) per wave
        if (ensure((void **)&c->d_fix, &c->fix_cap, (2 * groups + 64) * sizeof(uint64_t)) ||   // masks, first starts
            ensure((void **)&c->d_fixpos, &c->fixpos_cap, (groups * 64 + 64) * sizeof(uint64_t)))
            return DC_E_HIP;
        if (ensure((void **)&c->d_scr, &c->scr_cap, (size_t)D8_SCRATCH_WAVES * D8_WSCR)) return DC_E_HIP;
#define D8_LAUNCH(NW_, NC_)                                                                                   \
        LAUNCH(c, "huff_decode", (k_huff_decode8<NW_, NC_>), (tuples + NW_ - 1) / NW_ < 256 ? (tuples + NW_ - 1) / NW_ : 256, \
               NW_ * 64, d_words, bit_base, d_base, d_sync_base, d_sync_len, n, words, d_table, d_out, derr,       \
               c->d_queue, spct, (uint64_t *)c->d_fix, (uint64_t *)c->d_fixpos, (uint8_t *)c->d_scr)
#ifdef DC_AB_KERNELS
        if (c->opt_decode_variant == 1) {   // multi-symbol lookups, one group per wave
            LAUNCH(c, "huff_decode", k_huff_decode9<12>, groups < 256 * 12 ? (groups + 11) / 12 : 256, 12 * 64,
                   d_words, bit_base, d_base, d_sync_base, d_sync_len, n, words, d_table, d_out, derr, c->d_queue,
                   spct, (uint64_t *)c->d_fix, (uint64_t *)c->d_fixpos, (uint8_t *)c->d_scr);
        } else
#endif
        if (d_gexp) {   // (C5) with the symbols >= 0x80 per group
            LAUNCH(c, "huff_decode", (k_huff_decode8<11, 2, true>), (tuples + 10) / 11 < 256 ? (tuples + 10) / 11 : 256,
                   11 * 64, d_words, bit_base, d_base, d_sync_base, d_sync_len, n, words, d_table, d_out, derr,
                   c->d_queue, spct, (uint64_t *)c->d_fix, (uint64_t *)c->d_fixpos, (uint8_t *)c->d_scr, d_gexp);
        } else {   // one code per lookup, 11 waves x 2 chains (the 15-bit table takes 64 KiB of LDS)
            D8_LAUNCH(11, 2);
        }
#undef D8_LAUNCH
        c->last_groups = groups;
        LAUNCH(c, "huff_decode_fix", k_huff_decode8_fix, 256, D8F_WAVES * 64, d_words, n, words, d_table, d_out,
               derr, (const uint64_t *)c->d_fix, (const uint64_t *)c->d_fixpos, derr_next, d_gexp);
        return DC_OK;
    }
    const uint64_t wgs = (groups + DEC_WAVES - 1) / DEC_WAVES;
    const uint64_t grid = wgs < 256 ? wgs : 256;   // persistent: one 16-wave workgroup per CU
    LAUNCH(c, "huff_decode", k_huff_decode, grid, DEC_WAVES * 64, d_words, bit_base, d_base, d_sync_base, d_sync_len, S, n, d_table,
           d_out, derr, derr_next);
    return DC_OK;
}

int dc_huff_decode(dc_ctx *c, const uint32_t *d_words, uint64_t bit_base, uint64_t words,
                   const uint64_t *d_sync_base, const uint16_t *d_sync_len, uint32_t S, uint64_t n,
                   const dc_dtable *d_table, uint8_t *d_out)
{
    return decode_impl(c, d_words, bit_base, nullptr, words, d_sync_base, d_sync_len, S, n, d_table, d_out);
}

int dc_huff_decode_dev(dc_ctx *c, const uint32_t *d_words, const uint64_t *d_bit_base, uint64_t words,
                       const uint64_t *d_sync_base, const uint16_t *d_sync_len, uint32_t S, uint64_t n,
                       const dc_dtable *d_table, uint8_t *d_out)
{
    if (!d_bit_base) return DC_E_ARG;
    return decode_impl(c, d_words, 0, d_bit_base, words, d_sync_base, d_sync_len, S, n, d_table, d_out);
}

int dc_huff_decode_redo_count(dc_ctx *c, uint64_t *count)
{
    if (!c || !count) return DC_E_ARG;
    *count = 0;
    if (!c->d_fix || !c->last_groups) return DC_OK;
    uint64_t *h = (uint64_t *)malloc(c->last_groups * sizeof(uint64_t));
    if (!h) return DC_E_ARG;
    const bool ok = hipMemcpyAsync(h, c->d_fix, c->last_groups * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream) ==
                        hipSuccess &&
                    hipStreamSynchronize(c->stream) == hipSuccess;
    if (ok)
        for (uint64_t g = 0; g < c->last_groups; ++g) *count += (uint64_t)__builtin_popcountll(h[g]);
    free(h);
    return ok ? DC_OK : DC_E_HIP;
}

int dc_huff_decode_status(dc_ctx *c)
{
    int v = 0;
    HIPCHK(hipMemcpyAsync(&v, dec_err(c), sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return v ? DC_E_STREAM : DC_OK;
}

int dc_huff_text_bits(int format, int n_ary) { return text_bits(format, n_ary); }

int dc_huff_text(dc_ctx *c, const uint32_t *d_words, uint64_t bit_base, uint64_t bits, int format, int n_ary,
                 char *d_text, uint64_t *nchar)
{
    const int b = text_bits(format, n_ary);
    if (!c || b == 0 || (bits && (!d_words || !d_text))) return DC_E_ARG;
    const uint64_t nc = (bits + b - 1) / b;
    if (nchar) *nchar = nc;
    if (nc == 0) return DC_OK;
    LAUNCH(c, "text", k_text, (nc + 255) / 256, 256, d_words, bit_base, bits, format, n_ary, b, d_text);
    return DC_OK;
}

int dc_huff_text_parse(dc_ctx *c, const char *d_text, uint64_t nchar, int format, int n_ary, uint64_t bits,
                       uint32_t *d_words)
{
    const int b = text_bits(format, n_ary);
    if (!c || b == 0 || nchar * (uint64_t)b < bits || (bits && (!d_text || !d_words))) return DC_E_ARG;
    HIPCHK(hipMemsetAsync(c->d_err + 8, 0, sizeof(int), c->stream));
    const uint64_t nw = (bits + 31) / 32;
    if (nw == 0) return DC_OK;
    LAUNCH(c, "text_parse", k_text_parse, (nw + 255) / 256, 256, (const uint8_t *)d_text, nchar, format, n_ary, b,
           bits, d_words, c->d_err + 8);
    return DC_OK;
}

int dc_huff_text_parse_status(dc_ctx *c)
{
    if (!c) return DC_E_ARG;
    int v = 0;
    HIPCHK(hipMemcpyAsync(&v, c->d_err + 8, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return v ? DC_E_STREAM : DC_OK;
}

int dc_huff_base64url(dc_ctx *c, const uint32_t *d_words, uint64_t bit_base, uint64_t bits, char *d_text)
{
    if (!c || (bits && (!d_words || !d_text))) return DC_E_ARG;
    const uint64_t nchar = (bits + 5) / 6;
    if (nchar == 0) return DC_OK;
    LAUNCH(c, "base64url", k_base64url, (nchar + 255) / 256, 256, d_words, bit_base, bits, d_text);
    return DC_OK;
}

}  // extern "C"

// ---- byte-stream transducer codecs --------------------------------------------------
// tiles + scan (from state aux.s_init) + write; h_plan (optional) gets the whole composition
// (c0, c1, s0, s1) for shard plans; write = false stops after the scan
// gexp (M_SMALL_DEC only, dc_small_huff_decode): the tile summaries from the decoder's counts
// (k_small_dec_summ) instead of the counting pass
template <int M>
static int fsm_run(dc_ctx *c, const uint8_t *d_in, uint64_t len, uint64_t nelem, uint8_t *d_out, uint64_t *h_len,
                   const char *name, FsmAux aux = FsmAux{nullptr, 0, 0, 1, 1}, uint64_t *h_plan = nullptr,
                   bool write = true, const uint32_t *gexp = nullptr, uint64_t ngroups = 0, bool summ_ready = false)
{
    const uint64_t ntiles = SmMode<M>::fast ? sm_ntiles<M>(d_in, FsmOff<M>::v, nelem) : (nelem + FSM_TILE - 1) / FSM_TILE;
    const uint64_t nt = ntiles ? ntiles : 1;
    const uint64_t ng = (nt + FSM_GROUP - 1) / FSM_GROUP;
    if (ensure((void **)&c->d_summ, &c->summ_cap, (nt + ng) * sizeof(uint4))) return DC_E_HIP;
    if (ensure((void **)&c->d_entry, &c->entry_cap, ng * sizeof(uint64_t))) return DC_E_HIP;
    uint4 *gsum = c->d_summ + nt;
    if (ntiles == 0) {
        // empty: count 0, state unchanged; composition = identity
        c->h_pinned[0] = 0; c->h_pinned[1] = aux.s_init;
        c->h_pinned[2] = 0; c->h_pinned[3] = 0; c->h_pinned[4] = 0; c->h_pinned[5] = 1;
        HIPCHK(hipMemcpyAsync(c->d_meta, c->h_pinned, 6 * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
        c->h_pinned[6] = aux.s_init;
        HIPCHK(hipMemcpyAsync(c->d_entry, c->h_pinned + 6, sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
        uint32_t *idn = reinterpret_cast<uint32_t *>(c->h_pinned + 8);   // identity local composition
        idn[0] = 0; idn[1] = 0; idn[2] = 0; idn[3] = 1;
        HIPCHK(hipMemcpyAsync(c->d_summ, idn, sizeof(uint4), hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    } else {
        if (M == M_SMALL_DEC && gexp)
            LAUNCH(c, "small_dec_summ", k_small_dec_summ, (ntiles + 255) / 256, 256, gexp, ngroups, d_in, len, ntiles,
                   c->d_summ, c->d_meta);
        else if constexpr (SmMode<M>::fast) LAUNCH(c, name, k_small_tiles<M>, ntiles, 256, d_in, len, nelem, c->d_summ);
        else if (M == M_NYB_ENC && aux.frec && !summ_ready) return DC_E_STATE;   // (ranks with unsettled first touches)
        else if (summ_ready) {   // (k_mtf_resolve's: the scan below rewrites d_summ in place)
            if (!c->summ_fresh)
                HIPCHK(hipMemcpyAsync(c->d_summ, c->d_fraw, ntiles * sizeof(uint4), hipMemcpyDeviceToDevice, c->stream));
        }
        else if ((M == M_NYB_ENC && !aux.rk) || M == M_NYB_DEC || M == M_NYB_DBODY)
            LAUNCH(c, name, k_nyb_tiles<M == M_NYB_DEC ? M_NYB_DEC : M == M_NYB_DBODY ? M_NYB_DBODY : M_NYB_ENC>,
                   (ntiles + 4 * NYB_TPW - 1) / (4 * NYB_TPW), 256, d_in, len, nelem, ntiles, c->d_summ);
        else LAUNCH(c, name, k_fsm_tiles<M>, ntiles, 256, d_in, len, nelem, c->d_summ, aux);
        c->summ_fresh = false;   // (d_summ rewritten in place: no longer the resolver's summaries)
        LAUNCH(c, "fsm_scan_up", k_fsm_scan_up, ng, FSM_GROUP, c->d_summ, ntiles, gsum);
        LAUNCH(c, "fsm_scan", k_fsm_scan, 1, 1024, (const uint4 *)gsum, ng, c->d_entry, c->d_meta, aux.s_init);
    }
    if (write) {
        const uint64_t wgrid = ntiles ? ntiles : 1;
        if constexpr (SmMode<M>::fast)
            LAUNCH(c, SmMode<M>::dec ? "small_dec_write" : "small_write", k_small_write<M>, wgrid, SmMode<M>::wthreads, d_in, len, nelem, (const uint64_t *)c->d_entry,
                   (const uint4 *)c->d_summ, (const uint64_t *)c->d_meta, d_out);
        else if (M == M_NYB_ENC && !aux.rk && ntiles && !((uintptr_t)d_in & 15) && !c->opt_nyb_wtile_off)
            LAUNCH(c, FsmMode<M>::wname, k_nyb_enc_wtile<false>, (ntiles + 3) / 4, 256, d_in, len, nelem, ntiles,
                   (const uint64_t *)c->d_entry, (const uint4 *)c->d_summ, (const uint64_t *)c->d_meta, d_out, aux);
        else if (M == M_NYB_ENC && aux.rk && ntiles && !((uintptr_t)d_in & 15) && !((uintptr_t)aux.rk & 15) &&
                 !c->opt_nyb_wtile_off)
            LAUNCH(c, FsmMode<M>::wname, k_nyb_enc_wtile<true>, (ntiles + 3) / 4, 256, d_in, len, nelem, ntiles,
                   (const uint64_t *)c->d_entry, (const uint4 *)c->d_summ, (const uint64_t *)c->d_meta, d_out, aux);
        else if (M == M_NYB_DEC && ntiles && !((uintptr_t)d_in & 15) && !c->opt_nyb_wtile_off)
            LAUNCH(c, FsmMode<M>::wname, k_nyb_dec_wtile, (ntiles + 3) / 4, 256, d_in, len, nelem, ntiles,
                   (const uint64_t *)c->d_entry, (const uint4 *)c->d_summ, d_out, aux);
        else
            LAUNCH(c, FsmMode<M>::wname, k_fsm_write<M>, wgrid, 256, d_in, len, nelem, (const uint64_t *)c->d_entry,
                   (const uint4 *)c->d_summ, (const uint64_t *)c->d_meta, d_out, aux);
    }
    HIPCHK(hipMemcpyAsync(c->h_pinned, c->d_meta, 9 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (gexp && c->h_pinned[8] != 8) return DC_E_STREAM;   // (dc_small_huff_decode: not a type-8 stream)
    if (h_plan) for (int k = 0; k < 4; ++k) h_plan[k] = c->h_pinned[2 + k];
    c->fsm_in = write ? nullptr : d_in; c->fsm_len = len; c->fsm_nelem = nelem; c->fsm_mode = M;
    const bool nyb = M == M_NYB_ENC;
    const bool enc = FsmMode<M>::enc || (nyb && aux.whole);
    const uint64_t body = nyb ? c->h_pinned[0] + (aux.is_last ? c->h_pinned[1] : 0) : c->h_pinned[0];
    uint64_t total = (FsmMode<M>::body || (nyb && !aux.whole)) ? body : enc ? 2 + body : 1 + body;
    if (enc && total >= len) total = len + 1;
    if (h_len) *h_len = total;
    return DC_OK;
}

// the write pass alone, on the tile summaries and entries the last fsm_run(write = false) of
// the same input left in the context (a shard body sized before its output is placed)
template <int M>
static int fsm_write_planned(dc_ctx *c, const uint8_t *d_in, uint64_t len, uint64_t nelem, uint8_t *d_out,
                             uint64_t *h_len, FsmAux aux = FsmAux{nullptr, 0, 0, 1, 1})
{
    if (c->fsm_in != d_in || c->fsm_len != len || c->fsm_nelem != nelem || c->fsm_mode != M) return DC_E_STATE;
    const uint64_t ntiles = SmMode<M>::fast ? sm_ntiles<M>(d_in, FsmOff<M>::v, nelem) : (nelem + FSM_TILE - 1) / FSM_TILE;
    if constexpr (SmMode<M>::fast)
        LAUNCH(c, SmMode<M>::dec ? "small_dec_write" : "small_write", k_small_write<M>, ntiles ? ntiles : 1, SmMode<M>::wthreads, d_in, len, nelem,
               (const uint64_t *)c->d_entry, (const uint4 *)c->d_summ, (const uint64_t *)c->d_meta, d_out);
    else if (M == M_NYB_ENC && !aux.rk && ntiles && !((uintptr_t)d_in & 15) && !c->opt_nyb_wtile_off)
        LAUNCH(c, FsmMode<M>::wname, k_nyb_enc_wtile<false>, (ntiles + 3) / 4, 256, d_in, len, nelem, ntiles,
               (const uint64_t *)c->d_entry, (const uint4 *)c->d_summ, (const uint64_t *)c->d_meta, d_out, aux);
    else
        LAUNCH(c, FsmMode<M>::wname, k_fsm_write<M>, ntiles ? ntiles : 1, 256, d_in, len, nelem, (const uint64_t *)c->d_entry,
               (const uint4 *)c->d_summ, (const uint64_t *)c->d_meta, d_out, aux);
    HIPCHK(hipMemcpyAsync(c->h_pinned, c->d_meta, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->fsm_in = nullptr;
    if (h_len) *h_len = c->h_pinned[0];
    return DC_OK;
}

// the per-tile record counts of the last mtf_run(ranks)
static const uint2 *mtf_heads(const dc_ctx *c, uint64_t)
{
    return c->d_mhead;
}

// Adaptive nybble ranks (k_mtf_* pipeline) of elements 1..len-1 of d_in into c->d_rk, from the
// entry lists h_init. ranks = false: only the composition of the whole input from h_init
// into *h_final (a shard summary when h_init is empty).
static int mtf_run(dc_ctx *c, const uint8_t *d_in, uint64_t len, const MtfSum *h_init, bool ranks, MtfSum *h_final)
{
    const uint64_t n0 = len > 1 ? (len - 2) / MTF_TILE + 1 : 0;
    if (n0 == 0) {
        if (h_final) *h_final = *h_init;
        c->rk_in = d_in; c->rk_len = len;
        return DC_OK;
    }
    uint64_t nl[8], off[8];
    int levels = 0;
    uint64_t tot = 0;
    for (uint64_t n = n0;; n = (n + MTF_FAN - 1) / MTF_FAN) {
        nl[levels] = n; off[levels] = tot; tot += n; ++levels;
        if (n <= MTF_FAN) break;
    }
    // layout: [summaries, all levels][entries, all levels][init][final]
    if (ensure((void **)&c->d_mtf, &c->mtf_cap, (2 * tot + 2) * sizeof(MtfSum))) return DC_E_HIP;
    MtfSum *S = c->d_mtf, *E = c->d_mtf + tot, *init = c->d_mtf + 2 * tot, *fin = init + 1;
    // the entry lists through a pinned copy: no wait here (the stream is idle at every call: the
    // calls that follow an mtf_run end by reading back on it)
    if (!c->h_mtf && hipHostMalloc((void **)&c->h_mtf, sizeof(MtfSum), 0) != hipSuccess) return DC_E_HIP;
    memcpy(c->h_mtf, h_init, sizeof(MtfSum));
    HIPCHK(hipMemcpyAsync(init, c->h_mtf, sizeof(MtfSum), hipMemcpyHostToDevice, c->stream));
    if (ranks && ensure((void **)&c->d_rk, &c->rk_cap, ((len + 3) & ~3ull))) return DC_E_HIP;
    if (ranks && (ensure((void **)&c->d_mrec, &c->mrec_cap, n0 * 2 * MTF_REC * sizeof(uint4)) ||
                  ensure((void **)&c->d_mhead, &c->mhead_cap, n0 * sizeof(uint2)) ||
                  ensure((void **)&c->d_fraw, &c->fraw_cap, n0 * sizeof(uint4))))
        return DC_E_HIP;
    uint4 *const mrec = c->d_mrec;
    uint2 *const mhead = c->d_mhead;
    // a tile's elements start (1 + d_in % 16) % 16 bytes into its first granule: within its first
    // dword for the usual 16-B aligned input (k_mtf_walk<0/2>, no dword selects), anywhere (<1/3>)
    const bool gen = (((uintptr_t)d_in + 1) & 15u) >= 4u;
    if (ranks && !gen)   // the summaries, the ranks but for the first touches, and their list: one walk
        LAUNCH(c, "mtf_tiles", k_mtf_walk<2>, (n0 + 255) / 256, 256, d_in, len, n0, S, c->d_rk, mrec, mhead);
    else if (ranks)
        LAUNCH(c, "mtf_tiles", k_mtf_walk<3>, (n0 + 255) / 256, 256, d_in, len, n0, S, c->d_rk, mrec, mhead);
    else if (!gen)
        LAUNCH(c, "mtf_tiles", k_mtf_walk<0>, (n0 + 255) / 256, 256, d_in, len, n0, S, (uint8_t *)nullptr,
               (uint4 *)nullptr, (uint2 *)nullptr);
    else
        LAUNCH(c, "mtf_tiles", k_mtf_walk<1>, (n0 + 255) / 256, 256, d_in, len, n0, S, (uint8_t *)nullptr,
               (uint4 *)nullptr, (uint2 *)nullptr);
    for (int l = 0; l + 1 < levels; ++l)
        LAUNCH(c, "mtf_reduce", k_mtf_reduce, (nl[l + 1] * 16 + 255) / 256, 256, (const MtfSum *)(S + off[l]), nl[l],
               S + off[l + 1]);
    for (int l = levels - 1; l >= 0; --l) {
        const MtfSum *pe = (l == levels - 1) ? init : E + off[l + 1];
        const uint64_t groups = (nl[l] + MTF_FAN - 1) / MTF_FAN;
        LAUNCH(c, "mtf_down", k_mtf_down, (groups * 16 + 255) / 256, 256, (const MtfSum *)(S + off[l]), nl[l], pe,
               E + off[l], l == levels - 1 ? fin : (MtfSum *)nullptr);
    }
    if (ranks) {   // and the nybble encoder's tile summaries (fsm_run(..., summ_ready)): its tiles are these
        const uint64_t ng = (n0 + FSM_GROUP - 1) / FSM_GROUP;
        if (ensure((void **)&c->d_summ, &c->summ_cap, (n0 + ng) * sizeof(uint4))) return DC_E_HIP;
        LAUNCH(c, "mtf_ranks", k_mtf_resolve, (n0 + 255) / 256, 256, len, n0, (const MtfSum *)E, mrec,
               (const uint2 *)mhead, c->d_rk, c->d_fraw, c->d_summ);
        c->summ_fresh = true;
    }
    if (h_final) {
        HIPCHK(hipMemcpyAsync(h_final, fin, sizeof(MtfSum), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    c->rk_in = ranks ? d_in : nullptr; c->rk_len = len;
    return DC_OK;
}

// The adaptive decode's resolve (k_nyb_resolve_c) over the tokens in out[1, n), in segments
// of ADEC_SEG tokens (a control dword each).
#define ADEC_SEG (16ull << 20)
static int adec_fast(dc_ctx *c, uint8_t *d_out, uint64_t n)
{
    const uint64_t seg = std::min<uint64_t>(n - 1, ADEC_SEG);
    if (ensure((void **)&c->d_actl, &c->actl_cap, (seg + 64) * sizeof(uint32_t))) return DC_E_HIP;
    if (!c->d_astate && hipMalloc(&c->d_astate, 64 * sizeof(uint32_t)) != hipSuccess) return DC_E_HIP;
    for (uint64_t k0 = 1; k0 < n; k0 += ADEC_SEG) {
        const uint64_t k1 = std::min<uint64_t>(k0 + ADEC_SEG, n);
        const uint64_t grid = std::min<uint64_t>((k1 - k0 + 255) / 256, 8192);
        LAUNCH(c, "nyb_adec_ctl", k_nyb_adec_ctl, grid, 256, (const uint8_t *)d_out, k0, k1, n, c->d_actl);
        LAUNCH(c, "nyb_resolve", k_nyb_resolve_c, 1, 64, d_out, k0, k1, (const uint32_t *)c->d_actl, c->d_astate,
               k0 == 1 ? 1 : 0);
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    return DC_OK;
}

static MtfSum mtf_initial()   // initialize_dictionary (nybble_compression.c:546-562)
{
    MtfSum s;
    uint64_t L = 0;
    const char *init = " etaoins";
    for (int k = 0; k < 8; ++k) L |= (uint64_t)(uint8_t)init[k] << (8 * k);
    for (int q = 0; q < 16; ++q) { s.L[q] = L; s.cnt[q] = 8; }
    return s;
}

static int read_byte(dc_ctx *c, const uint8_t *d, uint8_t *v)
{
    HIPCHK(hipMemcpyAsync(c->h_pinned, d, 1, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    *v = *(uint8_t *)c->h_pinned;
    return DC_OK;
}

static int write_byte(dc_ctx *c, uint8_t *d, uint8_t v)
{
    HIPCHK(hipMemsetAsync(d, v, 1, c->stream));
    return DC_OK;
}

// decoder type dispatch shared by nybble and small (:744, :799, :806)
static int copy_typed(dc_ctx *c, const uint8_t *d_in, uint64_t m, uint8_t type, uint8_t *d_out, uint64_t *h_len,
                      bool *handled)
{
    *handled = true;
    if (type == ' ') {
        if (m > 1) HIPCHK(hipMemcpyAsync(d_out, d_in + 1, m - 1, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        *h_len = m - 1;
        return DC_OK;
    }
    *handled = false;
    return DC_OK;
}

extern "C" {

int dc_nyb_compress(dc_ctx *c, const uint8_t *d_in, uint64_t n, int modify, uint8_t *d_out, uint64_t *h_len)
{
    if (!c || !d_out || !h_len || (n && !d_in)) return DC_E_ARG;
    if (n == 0) { int r = write_byte(c, d_out, ' '); if (r) return r; HIPCHK(hipStreamSynchronize(c->stream)); *h_len = 1; return DC_OK; }
    if (!modify) return fsm_run<M_NYB_ENC>(c, d_in, n, n - 1, d_out, h_len, "nyb_enc_tiles");
    const MtfSum init = mtf_initial();
    int r = mtf_run(c, d_in, n, &init, true, nullptr);
    if (r) return r;
    // (the tile summaries: k_mtf_resolve's, when there are ranks)
    return fsm_run<M_NYB_ENC>(c, d_in, n, n - 1, d_out, h_len, "nyb_enca_tiles",
                              FsmAux{n > 1 ? c->d_rk : nullptr, 0, 0, 1, 1, 0, c->d_mrec, mtf_heads(c, n)}, nullptr, true,
                              nullptr, 0, n > 1);
}

// ---- chunked nybble container (DCNK) ---------------------------------------------------
uint64_t dc_nyb_chunked_bound(uint64_t n, uint32_t K)
{
    const uint64_t nch = (n && K) ? (n + K - 1) / K : 0;
    return NYBK_HEAD + 8 * (nch + 1) + n + 2 * nch;
}

int dc_nyb_compress_chunked(dc_ctx *c, const uint8_t *d_in, uint64_t n, int modify, uint32_t K, uint8_t *d_out,
                            uint64_t out_cap, uint64_t *h_len)
{
    if (!c || !d_out || !h_len || (n && !d_in) || K < 16 || ((uintptr_t)d_out & 7)) return DC_E_ARG;
    const uint64_t nch = n ? (n + K - 1) / K : 0;
    const uint64_t head = NYBK_HEAD + 8 * (nch + 1);
    if (out_cap < head) return DC_E_CAPACITY;
    uint32_t *h = (uint32_t *)c->h_pinned;
    h[0] = NYBK_MAGIC; h[1] = 1; h[2] = modify ? 1 : 0; h[3] = K;
    c->h_pinned[2] = n; c->h_pinned[3] = nch;
    HIPCHK(hipMemcpyAsync(d_out, c->h_pinned, NYBK_HEAD, hipMemcpyHostToDevice, c->stream));
    uint64_t *off = (uint64_t *)(d_out + NYBK_HEAD);
    if (nch == 0) {
        HIPCHK(hipMemsetAsync(off, 0, 8, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        *h_len = head;
        return DC_OK;
    }
    if (ensure((void **)&c->d_kscr, &c->kscr_cap, nch * ((uint64_t)K + 2))) return DC_E_HIP;
    if (ensure((void **)&c->d_klens, &c->klens_cap, nch * sizeof(uint64_t))) return DC_E_HIP;
    LAUNCH(c, "nyb_chunk_enc", k_nyb_chunk_enc, (nch + 63) / 64, 64, d_in, n, K, nch, modify ? 1 : 0, c->d_kscr,
           c->d_klens);
    LAUNCH(c, "nyb_chunk_scan", k_scan_u64, 1, 1024, (const uint64_t *)c->d_klens, nch, off);
    HIPCHK(hipMemcpyAsync(c->h_pinned, off + nch, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const uint64_t total = c->h_pinned[0];
    if (out_cap < head + total) return DC_E_CAPACITY;
    LAUNCH(c, "nyb_chunk_copy", k_nyb_chunk_copy, nch, 256, (const uint8_t *)c->d_kscr, K, (const uint64_t *)off,
           d_out + head);
    HIPCHK(hipStreamSynchronize(c->stream));
    *h_len = head + total;
    return DC_OK;
}

int dc_nyb_chunked_info(dc_ctx *c, const uint8_t *d_in, uint64_t m, uint64_t *h_n, int *h_modify, uint32_t *h_K)
{
    if (!c || !d_in || m < NYBK_HEAD) return DC_E_ARG;
    HIPCHK(hipMemcpyAsync(c->h_pinned, d_in, NYBK_HEAD, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const uint32_t *h = (const uint32_t *)c->h_pinned;
    if (h[0] != NYBK_MAGIC || h[1] != 1 || h[3] < 16) return DC_E_STREAM;
    if (h_n) *h_n = c->h_pinned[2];
    if (h_modify) *h_modify = (int)h[2];
    if (h_K) *h_K = h[3];
    return DC_OK;
}

int dc_nyb_decompress_chunked(dc_ctx *c, const uint8_t *d_in, uint64_t m, uint8_t *d_out, uint64_t out_cap,
                              uint64_t *h_len)
{
    if (!c || !d_out || !h_len || !d_in || ((uintptr_t)d_in & 7)) return DC_E_ARG;
    uint64_t n = 0;
    int modify = 0;
    uint32_t K = 0;
    int r = dc_nyb_chunked_info(c, d_in, m, &n, &modify, &K);
    if (r) return r;
    const uint64_t nch = c->h_pinned[3];
    if (nch != (n ? (n + K - 1) / K : 0) || m < NYBK_HEAD + 8 * (nch + 1)) return DC_E_STREAM;
    if (out_cap < n) return DC_E_CAPACITY;
    *h_len = n;
    if (nch == 0) return DC_OK;
    const uint64_t head = NYBK_HEAD + 8 * (nch + 1);
    uint64_t *err = c->d_meta + 8;
    HIPCHK(hipMemsetAsync(err, 0, 8, c->stream));
    LAUNCH(c, "nyb_chunk_dec", k_nyb_chunk_dec, (nch + 63) / 64, 64, d_in + head,
           (const uint64_t *)(d_in + NYBK_HEAD), m - head, n, K, nch, modify, d_out, err);
    HIPCHK(hipMemcpyAsync(c->h_pinned, err, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return c->h_pinned[0] ? DC_E_STREAM : DC_OK;
}

int dc_nyb_decompress_batch(dc_ctx *c, const uint8_t *d_in, const uint64_t *d_in_off, uint64_t count, int modify,
                            uint8_t *d_out, uint64_t out_cap, uint64_t *d_out_off, uint64_t *h_total)
{
    if (!c || !d_in_off || !d_out_off || !h_total || (count && !d_in)) return DC_E_ARG;
    *h_total = 0;
    if (count == 0) {
        HIPCHK(hipMemsetAsync(d_out_off, 0, sizeof(uint64_t), c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        return DC_OK;
    }
    if (ensure((void **)&c->d_klens, &c->klens_cap, count * sizeof(uint64_t))) return DC_E_HIP;
    uint64_t *err = c->d_meta + 8;
    HIPCHK(hipMemsetAsync(err, 0, 8, c->stream));
    const uint64_t grid = (count + 63) / 64;
    LAUNCH(c, "nyb_batch_len", k_nyb_batch_len, grid, 64, d_in, d_in_off, count, c->d_klens, err);
    LAUNCH(c, "nyb_batch_scan", k_scan_u64, 1, 1024, (const uint64_t *)c->d_klens, count, d_out_off);
    HIPCHK(hipMemcpyAsync(c->h_pinned, d_out_off + count, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(c->h_pinned + 1, err, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const uint64_t total = c->h_pinned[0];
    if (c->h_pinned[1]) return DC_E_ARG;
    *h_total = total;
    if (total > out_cap || (total && !d_out)) return DC_E_CAPACITY;
    LAUNCH(c, "nyb_batch_dec", k_nyb_batch_dec, grid, 64, d_in, d_in_off, (const uint64_t *)d_out_off, count, modify,
           d_out, err);
    HIPCHK(hipMemcpyAsync(c->h_pinned, err, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return c->h_pinned[0] ? DC_E_STREAM : DC_OK;
}

// ---- nybble shard bodies (dist.ShardedNybble) ---------------------------
int dc_nyb_mtf_summary(dc_ctx *c, const uint8_t *d_in, uint64_t len, uint8_t *h_lists, uint8_t *h_cnt)
{
    if (!c || !h_lists || !h_cnt || (len && !d_in)) return DC_E_ARG;
    MtfSum empty, fin;
    memset(&empty, 0, sizeof(empty));
    int r = mtf_run(c, d_in, len, &empty, false, &fin);
    if (r) return r;
    memcpy(h_lists, fin.L, 128);
    memcpy(h_cnt, fin.cnt, 16);
    return DC_OK;
}

static int lists_in(const uint8_t *h_lists, MtfSum *s)
{
    memcpy(s->L, h_lists, 128);
    for (int q = 0; q < 16; ++q) s->cnt[q] = 8;
    return DC_OK;
}

int dc_nyb_body_plan(dc_ctx *c, const uint8_t *d_in, uint64_t len, int modify, const uint8_t *h_lists,
                     uint64_t *h_plan)
{
    if (!c || !h_plan || !d_in || len < 1 || (modify && !h_lists)) return DC_E_ARG;
    FsmAux aux{nullptr, 0, 0, 0, 0};
    if (modify) {
        MtfSum init;
        lists_in(h_lists, &init);
        int r = mtf_run(c, d_in, len, &init, true, nullptr);
        if (r) return r;
        aux.rk = len > 1 ? c->d_rk : nullptr;
        aux.frec = c->d_mrec;
        aux.fhead = mtf_heads(c, len);
    }
    int r = fsm_run<M_NYB_ENC>(c, d_in, len, len - 1, nullptr, nullptr, "nyb_body_tiles", aux, h_plan, false,
                               nullptr, 0, modify && len > 1);
    if (r) return r;
    // rank of the last element (the byte a pending nybble of this shard belongs to)
    uint8_t last = 0xFF;
    if (len > 1) {
        if (modify) HIPCHK(hipMemcpyAsync(c->h_pinned, c->d_rk + (len - 2), 1, hipMemcpyDeviceToHost, c->stream));
        else HIPCHK(hipMemcpyAsync(c->h_pinned, d_in + (len - 1), 1, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        last = *(uint8_t *)c->h_pinned;
        if (!modify) {
            const char *t = " etaoins";
            const uint8_t b = last;
            last = 0xFF;
            for (int k = 0; k < 8; ++k) if ((uint8_t)t[k] == b) { last = (uint8_t)k; break; }
        }
    }
    h_plan[4] = last;
    return DC_OK;
}

int dc_nyb_body_write(dc_ctx *c, const uint8_t *d_in, uint64_t len, int modify, int pend_rank, int is_last,
                      uint8_t *d_out, uint64_t *h_len, int *h_state_out)
{
    if (!c || !d_out || !h_len || !d_in || len < 1 || pend_rank > 7) return DC_E_ARG;
    if (modify && len > 1 && (c->rk_in != d_in || c->rk_len != len)) return DC_E_ARG;   // plan this input first
    // the first-touch records only with ranks (an earlier adaptive call leaves d_mrec set: a
    // static body passing it would trip fsm_run's unsettled-ranks guard)
    const bool adaptive = modify && len > 1;
    FsmAux aux{adaptive ? c->d_rk : nullptr, pend_rank < 0 ? 0u : (uint32_t)pend_rank,
               pend_rank < 0 ? 0u : 1u, is_last ? 1u : 0u, 0, 0, adaptive ? c->d_mrec : nullptr,
               adaptive ? mtf_heads(c, len) : nullptr};
    int r = fsm_run<M_NYB_ENC>(c, d_in, len, len - 1, d_out, h_len, "nyb_body_tiles", aux, nullptr, true, nullptr,
                               0, modify && len > 1);
    if (r) return r;
    if (h_state_out) *h_state_out = (int)c->h_pinned[1];
    return DC_OK;
}

int dc_nyb_dbody_plan(dc_ctx *c, const uint8_t *d_in, uint64_t len, uint64_t m, uint64_t *h_plan)
{
    if (!c || !h_plan || (m && !d_in) || m > len || len > m + 1) return DC_E_ARG;
    return fsm_run<M_NYB_DBODY>(c, d_in, len, m, nullptr, nullptr, "nyb_dbody_tiles", FsmAux{nullptr, 0, 0, 0, 0},
                                h_plan, false);
}

int dc_nyb_dbody_write(dc_ctx *c, const uint8_t *d_in, uint64_t len, uint64_t m, int s_in, uint8_t *d_out,
                       uint64_t *h_len, int *h_state_out)
{
    if (!c || !d_out || !h_len || (m && !d_in) || m > len || len > m + 1 || (s_in & ~1)) return DC_E_ARG;
    int r = fsm_run<M_NYB_DBODY>(c, d_in, len, m, d_out, h_len, "nyb_dbody_tiles",
                                 FsmAux{nullptr, 0, (uint32_t)s_in, 0, 0});
    if (r) return r;
    if (h_state_out) *h_state_out = (int)c->h_pinned[1];
    return DC_OK;
}

int dc_nyb_decompress(dc_ctx *c, const uint8_t *d_in, uint64_t m, int modify, uint8_t *d_out, uint64_t *h_len)
{
    if (!c || !d_out || !h_len || (m && !d_in)) return DC_E_ARG;
    if (m == 0) { *h_len = 0; return DC_OK; }
    uint8_t type = 0;
    int r = read_byte(c, d_in, &type);
    if (r) return r;
    if (type == 0xAF) {
        if (m < 2) { *h_len = 0; return DC_OK; }
        if (!modify) return fsm_run<M_NYB_DEC>(c, d_in, m, m - 2, d_out, h_len, "nyb_dec_tiles");
#ifdef DC_AB_KERNELS
        if (c->opt_adec_v1 == 1) {   // A/B only: the one-pass single-wave decoder
            LAUNCH(c, "nyb_adec", k_nyb_adec, 1, 64, d_in, m, d_out, c->d_meta);
            HIPCHK(hipMemcpyAsync(c->h_pinned, c->d_meta, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            *h_len = c->h_pinned[0];
            return DC_OK;
        }
#endif
        // tokens by the static transducer (parallel), then one wave resolves them in place
        r = fsm_run<M_NYB_DEC>(c, d_in, m, m - 2, d_out, h_len, "nyb_tok_tiles", FsmAux{nullptr, 0, 0, 1, 1, 1});
        if (r) return r;
        const uint64_t n = *h_len;
        if (n > 1 && c->opt_adec_v1 == 0) return adec_fast(c, d_out, n);   // control words + k_nyb_resolve_c
#ifdef DC_AB_KERNELS
        if (n > 1) {
            if (c->opt_adec_v1 == 2) LAUNCH(c, "nyb_resolve", k_nyb_resolve, 1, 64, d_out, n);   // A/B: r2's
            else LAUNCH(c, "nyb_resolve", k_nyb_resolve_s, 1, 64, d_out, n);
        }
#endif
        HIPCHK(hipStreamSynchronize(c->stream));
        return DC_OK;
    }
    bool handled = false;
    r = copy_typed(c, d_in, m, type, d_out, h_len, &handled);
    if (r || handled) return r;
    HIPCHK(hipMemcpyAsync(d_out, d_in, m, hipMemcpyDeviceToDevice, c->stream));   // unknown type (:806-812)
    HIPCHK(hipStreamSynchronize(c->stream));
    *h_len = m;
    return DC_OK;
}

int dc_small_compress(dc_ctx *c, const uint8_t *d_in, uint64_t n, uint8_t *d_out, uint64_t *h_len)
{
    if (!c || !d_out || !h_len || (n && !d_in)) return DC_E_ARG;
    if (n == 0) { int r = write_byte(c, d_out, ' '); if (r) return r; HIPCHK(hipStreamSynchronize(c->stream)); *h_len = 1; return DC_OK; }
    return fsm_run<M_SMALL_ENC>(c, d_in, n, n - 1, d_out, h_len, "small_enc_tiles");
}

int dc_small_compress_body(dc_ctx *c, const uint8_t *d_in, uint64_t len, int left_halo, uint64_t nelem,
                           uint8_t *d_out, uint64_t *h_len)
{
    if (!c || !d_out || !h_len || (len && !d_in) || (nelem && nelem + 1 > len)) return DC_E_ARG;
    if (nelem == 0) { *h_len = 0; return DC_OK; }
    return left_halo ? fsm_run<M_SMALL_BODY1>(c, d_in, len, nelem, d_out, h_len, "small_body_tiles")
                     : fsm_run<M_SMALL_BODY0>(c, d_in, len, nelem, d_out, h_len, "small_body_tiles");
}

int dc_small_compress_body_plan(dc_ctx *c, const uint8_t *d_in, uint64_t len, int left_halo, uint64_t nelem,
                                uint64_t *h_len)
{
    if (!c || !h_len || (len && !d_in) || (nelem && nelem + 1 > len)) return DC_E_ARG;
    if (nelem == 0) { c->fsm_in = nullptr; *h_len = 0; return DC_OK; }
    return left_halo ? fsm_run<M_SMALL_BODY1>(c, d_in, len, nelem, nullptr, h_len, "small_body_tiles",
                                              FsmAux{nullptr, 0, 0, 1, 1}, nullptr, false)
                     : fsm_run<M_SMALL_BODY0>(c, d_in, len, nelem, nullptr, h_len, "small_body_tiles",
                                              FsmAux{nullptr, 0, 0, 1, 1}, nullptr, false);
}

int dc_small_compress_body_write(dc_ctx *c, const uint8_t *d_in, uint64_t len, int left_halo, uint64_t nelem,
                                 uint8_t *d_out, uint64_t *h_len)
{
    if (!c || !d_out || !h_len || (len && !d_in) || (nelem && nelem + 1 > len)) return DC_E_ARG;
    if (nelem == 0) { *h_len = 0; return DC_OK; }
    return left_halo ? fsm_write_planned<M_SMALL_BODY1>(c, d_in, len, nelem, d_out, h_len)
                     : fsm_write_planned<M_SMALL_BODY0>(c, d_in, len, nelem, d_out, h_len);
}

int dc_small_decompress_body(dc_ctx *c, const uint8_t *d_in, uint64_t m, uint8_t *d_out, uint64_t *h_len)
{
    if (!c || !d_out || !h_len || (m && !d_in)) return DC_E_ARG;
    if (m == 0) { *h_len = 0; return DC_OK; }
    return fsm_run<M_SMALL_DBODY>(c, d_in, m, m, d_out, h_len, "small_dbody_tiles");
}

int dc_small_huff_decode(dc_ctx *c, const uint32_t *d_words, uint64_t bit_base, uint64_t words,
                         const uint64_t *d_sync_base, const uint16_t *d_sync_len, uint32_t S, uint64_t m,
                         const dc_dtable *d_table, uint8_t *d_m, uint8_t *d_out, uint64_t *h_len)
{
    if (!c || !d_m || !d_out || !h_len) return DC_E_ARG;
    // the counted path needs k_huff_decode8 (decode_impl's fast8 conditions; the A/B variant 1
    // decoder never writes the per-group counts): anything else runs the two stages as they are
    const bool counted = S == 64 && m >= 2 && !((uintptr_t)d_m & 15) && !c->opt_decode_general &&
                         c->opt_decode_variant == 0 && m < (1ull << 37) && words < (1ull << 31);
    if (!counted) {
        const int r = decode_impl(c, d_words, bit_base, nullptr, words, d_sync_base, d_sync_len, S, m, d_table, d_m);
        return r ? r : dc_small_decompress(c, d_m, m, d_out, h_len);
    }
    const uint64_t groups = dc_huff_sync_groups(m, 64);
    if (ensure((void **)&c->d_gexp, &c->gexp_cap, (groups + 2) * sizeof(uint32_t))) return DC_E_HIP;
    int r = decode_impl(c, d_words, bit_base, nullptr, words, d_sync_base, d_sync_len, 64, m, d_table, d_m, c->d_gexp);
    if (r) return r;
    r = fsm_run<M_SMALL_DEC>(c, d_m, m, m - 2, d_out, h_len, "small_dec_tiles", FsmAux{nullptr, 0, 0, 1, 1}, nullptr,
                             true, c->d_gexp, groups);
    if (r == DC_E_STREAM) return dc_small_decompress(c, d_m, m, d_out, h_len);   // not a type-8 stream
    return r;
}

int dc_small_decompress(dc_ctx *c, const uint8_t *d_in, uint64_t m, uint8_t *d_out, uint64_t *h_len)
{
    if (!c || !d_out || !h_len || (m && !d_in)) return DC_E_ARG;
    if (m == 0) { *h_len = 0; return DC_OK; }
    uint8_t type = 0;
    int r = read_byte(c, d_in, &type);
    if (r) return r;
    if (type == 8) {
        if (m < 2) { *h_len = 0; return DC_OK; }
        return fsm_run<M_SMALL_DEC>(c, d_in, m, m - 2, d_out, h_len, "small_dec_tiles");
    }
    bool handled = false;
    r = copy_typed(c, d_in, m, type, d_out, h_len, &handled);
    if (r || handled) return r;
    *h_len = 0;   // "invalid compressed data": empty output (small_compression.c:497-499)
    return DC_OK;
}

}  // extern "C"
