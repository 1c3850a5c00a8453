// gz_pvinc.hip -- incremental policy-value forward of a search's grandchildren, and
// the tree forward's classification kernels (AlphaZeroGomokuNet, neural_network.py:
// 74-159, f16x3 precision).
//
// MCTSNode.__init__ runs GomokuModel.predict for every new node (ai_agent.py:
// 522-523).  A root child differs from the root by one stone at cell m, so in
// layer L of the tower (x0 = conv0, y1, x1, y2, x2) only the positions within
// Chebyshev radius L+1 of m can differ from the root's maps: 3x3, 5x5, 7x7, 9x9,
// 11x11 squares (clipped to the board) -- about 31 % of the 4 x 225 positions of
// the residual convs.  The root is evaluated by the full kernel, which also stores
// its x0, y1, x1, y2 maps and its pre-BN accumulators (gz_pvnet.hip,
// pv_kernel_f16x3<.., true>).  The root children are computed as a delta of the
// root's accumulators by pv_dg_kernel (gz_pvdg.hip); a child with children of its
// own also stores its recomputed squares (its "patch").
//
// Grandchildren (a child of a root child, one more stone at m2): pv_sib_kernel below.
// Their windows are the root's maps overlaid with the parent's patch around the
// parent's stone; the recomputed positions (radius L+1 around m2) take the full
// kernel's products in the full kernel's order (k = tap*128 + cin in 32-deep MFMA
// k-steps, hi*hi, w_lo*a_hi, w_hi*a_lo; the same epilogue, hi/lo split and head-conv
// partial sums per wave).  Given the parent's patch they are the full forward's
// values; the patch itself carries the delta's rounding (tests/test_gpu_pvinc.py).
#include <hip/hip_runtime.h>
#include <type_traits>

#include <cstdlib>
#include <string>

#include "gz_f16conv.h"
#include "gz_pvnet.h"
#include "../../include/gzero.h"

using namespace gzpv;

namespace {

using namespace gzc;

// Phase stamps (tools/pvinc_bench.py only): -DGZ_PVINC_STAMPS accumulates s_memtime
// deltas of workgroup 0 / thread 0 per phase (vector atomics); compiled out otherwise.
#ifdef GZ_PVINC_STAMPS
__device__ unsigned long long gz_pvinc_stamps[32];  // [0, 16): pv_sib_kernel
__device__ unsigned long long gz_pvinc_stamps_n[2];
#endif
constexpr int P_X0 = 49, P_Y1 = 81, P_X1 = 121, P_Y2 = 169;  // window positions, radius 3..6
constexpr int wbytes(int P) { return 2 * 16 * P * 16; }       // hi + lo planes
constexpr int HP_ROWS = 128;                                  // >= 121 rows of the x2 square

// A window of a map: radius R around the child's stone (cr, cc), width w = 2R+1,
// P = w*w positions, hi plane then lo plane, each [16 cg][P][8].  The geometry is
// compile-time, so window addressing folds into instruction offsets and constant
// divisions.
template <int R>
struct Win {
    static constexpr int r = R, w = 2 * R + 1, P = w * w;
    _Float16* hi;
    __device__ static constexpr int plane() { return 16 * P * 8; }
    __device__ static constexpr int off(int ch0, int loc) { return ((ch0 >> 3) * P + loc) * 8 + (ch0 & 7); }
};

// the recomputed rows of one layer: the square of radius rl around (cr, cc),
// clipped, row-major
struct Rows {
    int r0, c0, wr, n;
};
__device__ inline Rows make_rows(int cr, int cc, int rl) {
    Rows q;
    q.r0 = cr - rl < 0 ? 0 : cr - rl;
    const int r1 = cr + rl > BN - 1 ? BN - 1 : cr + rl;
    q.c0 = cc - rl < 0 ? 0 : cc - rl;
    const int c1 = cc + rl > BN - 1 ? BN - 1 : cc + rl;
    q.wr = c1 - q.c0 + 1;
    q.n = (r1 - q.r0 + 1) * q.wr;
    return q;
}

template <int NMAX>
struct TilePos {
    int pr[NMAX], pc[NMAX], row[NMAX];
    bool valid[NMAX];
};

template <int NMAX, int R>
__device__ __forceinline__ void tile_positions(const Rows& rows, int t0, int lane, TilePos<NMAX>& tp) {
    const int pl = lane & 15;
    const float inv = 1.0f / (float)rows.wr;
#pragma unroll
    for (int m = 0; m < NMAX; m++) {
        int i = (t0 + m) * 16 + pl;
        tp.row[m] = i;
        tp.valid[m] = i < rows.n;
        if (i >= rows.n) i = (t0 + m) * 16;
        const int rr = (int)(((float)i + 0.5f) * inv);  // exact: i < 256, wr <= 11
        tp.pr[m] = rows.r0 + rr;
        tp.pc[m] = rows.c0 + (i - rr * rows.wr);
    }
}

template <int NMAX, class WI>
__device__ __forceinline__ void tile_centres(const TilePos<NMAX>& tp, int cr, int cc, int (&ctr)[NMAX]) {
#pragma unroll
    for (int m = 0; m < NMAX; m++) ctr[m] = (tp.pr[m] - cr + WI::r) * WI::w + (tp.pc[m] - cc + WI::r);
}

__device__ inline int bit_of_board(int r, int c) { return r * 16 + c; }

// A parent's patch for its grandchildren: the recomputed squares of its maps
// (x0 r1, y1 r2, x1 r3, y2 r4), [plane][16 cg][(2r+1)^2][8] each, in that order
constexpr int PATCH_OFF[4] = {0, 9 * 256, 34 * 256, 83 * 256};  // halves
constexpr int PATCH_HALVES = PV_PATCH_HALVES;


struct TreeArgs {
    const int32_t* cinfo;  // per leaf (tree_lists_kernel): -1, or (GC << 30) | (root map slot << 8) | stone cell
    const float* W;
    const uint32_t* boards;
    const int32_t* meta;
    const int32_t* ord;
    const int32_t* pslot;
    const _Float16* maps;
    _Float16* patches;
    float* hbuf;
    int32_t* tiles;  // 16-row MFMA tile-taps executed by the residual convs [children, grandchildren]
    int32_t* queue;  // [8] per-XCD chunk heads of pv_sib_kernel, zero at the launch
};

// ============================================================ sibling-batched incremental forward
// pv_sib_kernel: the same node computation as tree_node, scheduled so that one pass
// over a layer's weights serves several nodes.  tree_node streams each layer's 576 KB
// of hi/lo weight fragments from L2 once per node (twice on the pair layers) for 25-121
// output rows, which made pv_child_kernel bound by the L2 -> CU rate (3.86 MB per node,
// MFMA busy 0.44).  Here a workgroup takes a chunk of up to SIB_G consecutive nodes (a
// root's children are adjacent leaves, so a chunk usually shares one root) and runs the
// tower layer-major over the chunk:
//   y1: one pass over all 6 nodes (6 X0 r3 windows in LDS, up to 150 rows)
//   x1: two passes of 3 (Y1 r4 windows), y2: three passes of 2 (X1 r5), x2 + heads: 1 (Y2 r6)
// The rows of a pass are the nodes' recomputed squares packed back to back in 16-row
// M tiles (no per-node tile padding).  Each node's recomputed squares (x0 r1, y1 r2, x1
// r3, y2 r4: the patch layout) go to global memory between layers -- into its patch
// slot if it has grandchildren, else into the workgroup's scratch -- and the next
// layer's windows are filled from the root's maps overlaid with them.  Four waves, one
// per SIMD: wave np owns n-tiles {2np, 2np+1} over ALL M tiles of the pass, so each
// weight fragment is read once per pass and each activation fragment feeds 6 MFMAs.
// Weight bytes per node: 576 KB x (1/6 + 1/3 + 1/2 + 1) = 1.15 MB (was 3.7 MB).
// Every output element takes the full kernel's products in the full kernel's order
// (the full kernel's k-loop and epilogues), so results stay bitwise those of the full
// forward.  (Two waves per SIMD splitting the M tiles, reading each fragment twice,
// measured 1.5 % slower with the position-major fills.)
constexpr int NTS = 256, SIB_MH = 1;  // 4 waves; SIB_MH: M halves per n-tile pair
constexpr int sib_tiles(int t) { return t; }
constexpr int SIB_G = 6;
static_assert(SIB_G <= PV_SCRATCH_PATCHES, "tree scratch: one workgroup per grid entry");
constexpr int SIB_WIN = SIB_G * wbytes(P_X0);
static_assert(3 * wbytes(P_Y1) <= SIB_WIN && 2 * wbytes(P_X1) <= SIB_WIN && wbytes(P_Y2) <= SIB_WIN, "windows");
constexpr int SIB_HP = SIB_WIN;                     // head partials [4 pairs][3][HP_ROWS]
constexpr int SIB_U = SIB_HP + 4 * 3 * HP_ROWS * 4;  // unit table
constexpr int SIB_POS = SIB_U + SIB_G * 128;  // SibUnit: 128 B; then the chunk's first list entry
constexpr int LDS_S = SIB_POS + 16;
static_assert(LDS_S <= 160 * 1024, "LDS budget");

// phase stamps of pv_sib_kernel (workgroup 0, thread 0; -DGZ_PVINC_STAMPS builds only)
template <int BASE = 0>
struct SibStamp {
#ifdef GZ_PVINC_STAMPS
    unsigned long long t = __builtin_amdgcn_s_memtime();
    __device__ void operator()(int i) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();
            atomicAdd(&gz_pvinc_stamps[BASE + i], t_ - t);
            t = t_;
        }
    }
#else
    __device__ void operator()(int) {}
#endif
};

struct SibUnit {
    const _Float16* gm;   // the root's maps x0, y1, x1, y2
    _Float16* own;        // this node's recomputed squares (patch layout)
    const _Float16* par;  // grandchild: the parent's patch
    int leaf, base, cell, pcell;  // node, record base (root / parent), stone, parent's stone
    int pad[6];
    uint32_t board[16];   // the node's bit-plane board (conv0's input)
};
static_assert(sizeof(SibUnit) == 128, "unit size");

__device__ inline int iabs(int x) { return x < 0 ? -x : x; }

// Where map MAP (0..3 = x0, y1, x1, y2) holds on-board position (pr, pc) for unit u:
// the node's own recomputed square (radius MAP+1 around its stone), a grandchild's
// parent's square, else the root's map.  Channel c's hi value is at
// base + (c >> 3) * cs + (c & 7), its lo value lo halves further.
struct MapLoc {
    const _Float16* base;
    int cs, lo;
};
template <int MAP>
__device__ __forceinline__ MapLoc map_loc(const SibUnit& u, int pr, int pc) {
    constexpr int rc = MAP + 1, S = 2 * rc + 1, SS = S * S;
    const int cr = u.cell / BN, cc = u.cell - (u.cell / BN) * BN;
    MapLoc L;
    L.base = u.gm + MAP * PV_MAP_HALVES + (pr * BN + pc) * 8;
    L.cs = 256 * 8;
    L.lo = PV_MAP_PLANE;
    {  // the parent's square
        const int r1 = u.pcell / BN, c1 = u.pcell - (u.pcell / BN) * BN;
        if (iabs(pr - r1) <= rc && iabs(pc - c1) <= rc) {
            L.base = u.par + PATCH_OFF[MAP] + ((pr - r1 + rc) * S + (pc - c1 + rc)) * 8;
            L.cs = SS * 8;
            L.lo = 16 * SS * 8;
        }
    }
    if (iabs(pr - cr) <= rc && iabs(pc - cc) <= rc) {
        L.base = u.own + PATCH_OFF[MAP] + ((pr - cr + rc) * S + (pc - cc + rc)) * 8;
        L.cs = SS * 8;
        L.lo = 16 * SS * 8;
    }
    return L;
}

// Windows (radius R = MAP + 3) of map MAP for units [u0, u0 + ng) at LDS offset 0, one
// after another in the [plane][16 cg][P][8] layout: each position as map_loc places it, zeros
// (a zero source) off the board.  LDS-DMA (global_load_lds_dwordx4: item i of a unit's
// window lands at byte 16 i, wave-uniform base + 16 lane), so a fill holds no
// registers and all its loads are in flight at once; the caller's __syncthreads drains
// it.  Unit by unit, with the unit's fields in scalar registers.  The x0 windows (MAP
// 0) load the root's values at the node's own square too; conv0 overwrites them
// after the barrier.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
__device__ uint4 gz_sib_zero16[1];  // zero-initialised

// uniform copy of a unit's fields (SGPRs)
struct SibU {
    const _Float16 *gm, *own, *par;
    int cr, cc, r1, c1;
};
__device__ __forceinline__ const _Float16* rfl_ptr(const _Float16* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (const _Float16*)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ SibU sib_uniform(const SibUnit& u) {
    SibU s;
    s.gm = rfl_ptr(u.gm);
    s.own = rfl_ptr(u.own);
    s.par = rfl_ptr(u.par);
    const int cell = __builtin_amdgcn_readfirstlane(u.cell), pcell = __builtin_amdgcn_readfirstlane(u.pcell);
    s.cr = cell / BN;
    s.cc = cell - s.cr * BN;
    s.r1 = pcell / BN;
    s.c1 = pcell - s.r1 * BN;
    return s;
}

template <int MAP>
__device__ __forceinline__ void sib_fill(char* lds, const SibUnit* U, int u0, int ng, int tid) {
    constexpr int R = MAP + 3, Wd = 2 * R + 1, P = Wd * Wd, PER = 2 * 16 * P;
    constexpr int rc = MAP + 1, S = 2 * rc + 1, SS = S * S;
    // position-major: work blocks (unit, 64 window positions); a lane works out its
    // position's source once (root map, own square, parent's square or zero), then its
    // 32 channel-group planes go by LDS-DMA (for one plane a wave's positions are
    // contiguous in LDS; at the source the planes are a fixed stride apart).  (The
    // item-major fill, one 16-B item per thread, spent ~60 VALU per item: 136.7 vs
    // 141.0 ms per forward.)
    constexpr int NB = (P + 63) / 64;
    const int lane = tid & 63, wave = tid >> 6;
    for (int blk = wave; blk < ng * NB; blk += NTS / 64) {
        const int g = blk / NB, b0 = (blk - g * NB) * 64, loc = b0 + lane;
        const SibU u = sib_uniform(U[u0 + g]);
        const int dr = loc / Wd - R, dc = loc % Wd - R;
        const int pr = u.cr + dr, pc = u.cc + dc;
        const bool on = pr >= 0 && pr < BN && pc >= 0 && pc < BN;
        const bool own = on && iabs(dr) <= rc && iabs(dc) <= rc;
        const _Float16* src = (const _Float16*)gz_sib_zero16;
        int stride = 0;  // halves between channel-group planes at the source
        if (on) {
            src = u.gm + MAP * PV_MAP_HALVES + (pr * BN + pc) * 8;
            stride = 256 * 8;
        }
        if (MAP > 0 && own) {
            src = u.own + PATCH_OFF[MAP] + ((dr + rc) * S + (dc + rc)) * 8;
            stride = SS * 8;
        }
        if (on && !own && iabs(pr - u.r1) <= rc && iabs(pc - u.c1) <= rc) {
            src = u.par + PATCH_OFF[MAP] + ((pr - u.r1 + rc) * S + (pc - u.c1 + rc)) * 8;
            stride = SS * 8;
        }
        char* dst = lds + (size_t)g * PER * 16 + (size_t)b0 * 16;  // + lane * 16 by the DMA
        if (loc < P) {
#pragma unroll
            for (int pcg = 0; pcg < 32; pcg++)
                __builtin_amdgcn_global_load_lds((glb_void_t*)(src + pcg * stride), (lds_void_t*)(dst + pcg * P * 16), 16,
                                                 0, 0);
        }
    }
}

// The k-loop of a pass for the wave's n-tiles {nt0, nt0+1} over NT M tiles: the full kernel's
// k-steps, products and accumulation order, with one wave per SIMD: each tile's
// activation fragments for the next k-step are read right after its MFMAs (the other
// tiles' MFMAs cover the LDS latency), weight fragments 4 k-steps ahead.  act = the
// pass's windows (each [plane][16 cg][P][8]); ctr[m] = the lane's window-local row
// (unit offset included).
template <int NT, int NMAX, int R>
__device__ __forceinline__ void sib_conv_nt(const _Float16* act, const int (&ctr)[NMAX], const _Float16* __restrict__ Wf,
                                            int nt0, int lane, f32x4 (&acc)[2][NMAX]) {
    constexpr int Wd = 2 * R + 1, P = Wd * Wd, CQ = 4, KS = 9 * CQ, PLANE = 16 * P * 8;
    constexpr int KS_BYTES = 8 * 64 * 8 * 2, LO_BYTES = KS * KS_BYTES, RING = 4;
    static_assert(RING == 4, "ring depth");
    // Weight fragments 3 k-steps ahead: at the START of k-step j, k-step j + 3 is loaded
    // into the slot k-step j - 1 has just released.  So at the tap loop's back-edge --
    // where the compiler waits for every outstanding load (vmcnt(0)) -- the newest
    // loads were issued a whole k-step of MFMAs earlier.
    const int q = lane >> 4;
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)Wf, 0, 0x7fffffff, 0x00020000);
    const int wo = (nt0 * 64 + lane) * 16;
    auto wload = [&](int ks, int n, int lo) -> h8 {
        return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, wo, ks * KS_BYTES + n * 1024 + lo * LO_BYTES, 0));
    };
    h8 b[RING][2][2];
#pragma unroll
    for (int c = 0; c < RING - 1; c++)
#pragma unroll
        for (int n = 0; n < 2; n++) {
            b[c][n][0] = wload(c, n, 0);
            b[c][n][1] = wload(c, n, 1);
        }
    // the accumulators as an exact-size local array (the caller's has NMAX entries):
    // keeps the register allocator from shuffling partial tuples inside the loop
    f32x4 c[2][NT];
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int m = 0; m < NT; m++) c[n][m] = acc[n][m];
    int nb[NT];
    h8 ah[NT], al[NT];
    int ctr_[NMAX];
#pragma unroll
    for (int m = 0; m < NMAX; m++) ctr_[m] = ctr[m];
#pragma unroll
    for (int m = 0; m < NT; m++) {
        nb[m] = (ctr_[m] - Wd - 1 + q * P) * 8;  // tap 0 = (-1, -1)
        ah[m] = *(const h8*)(act + nb[m]);
        al[m] = *(const h8*)(act + PLANE + nb[m]);
    }
#pragma unroll 1
    for (int tap = 0; tap < 9; tap++) {
        const int t2 = tap + 1 < 9 ? tap + 1 : 0;  // past the last tap: tap 0 again (unused)
        const int toff = (t2 / 3 - 1) * Wd + (t2 % 3 - 1);
#pragma unroll
        for (int cq = 0; cq < CQ; cq++) {
            const int sl = cq, sr = (cq + 3) & 3;
            {  // k-step ks + 3 into the slot of ks - 1 (past the end: the first k-steps again, unused)
                const int ksr = tap * CQ + cq + 3;
                const int kn = ksr < KS ? ksr : ksr - KS;
#pragma unroll
                for (int n = 0; n < 2; n++) {
                    b[sr][n][0] = wload(kn, n, 0);
                    b[sr][n][1] = wload(kn, n, 1);
                }
            }
#pragma unroll
            for (int m = 0; m < NT; m++) {
#pragma unroll
                for (int n = 0; n < 2; n++)
                    c[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[sl][n][0], ah[m], c[n][m], 0, 0, 0);
#pragma unroll
                for (int n = 0; n < 2; n++)
                    c[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[sl][n][1], ah[m], c[n][m], 0, 0, 0);
#pragma unroll
                for (int n = 0; n < 2; n++)
                    c[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[sl][n][0], al[m], c[n][m], 0, 0, 0);
                int o;
                if (cq < CQ - 1) {
                    o = nb[m] + (cq + 1) * 4 * P * 8;
                } else {
                    nb[m] = (ctr_[m] + toff + q * P) * 8;
                    o = nb[m];
                }
                ah[m] = *(const h8*)(act + o);
                al[m] = *(const h8*)(act + PLANE + o);
            }
            // pin the order (the default scheduler sinks each read to its use and then
            // waits for it there): the weight refill, then per tile its 6 MFMAs and its
            // 2 reads for the next k-step
            __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);  // VMEM read
#pragma unroll
            for (int m = 0; m < NT; m++) {
                __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);  // MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
            }
        }
    }
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int m = 0; m < NT; m++) acc[n][m] = c[n][m];
}

template <int NMAX, int R>
__device__ __forceinline__ void sib_conv(const _Float16* act, const int (&ctr)[NMAX], int nt, const _Float16* __restrict__ Wf,
                                         int nt0, int lane, f32x4 (&acc)[2][NMAX]) {
    static_assert(NMAX >= 1 && NMAX <= 12, "tile counts");
    switch (nt) {
        case 1: sib_conv_nt<1, NMAX, R>(act, ctr, Wf, nt0, lane, acc); break;
        case 2: if constexpr (NMAX >= 2) sib_conv_nt<2, NMAX, R>(act, ctr, Wf, nt0, lane, acc); break;
        case 3: if constexpr (NMAX >= 3) sib_conv_nt<3, NMAX, R>(act, ctr, Wf, nt0, lane, acc); break;
        case 4: if constexpr (NMAX >= 4) sib_conv_nt<4, NMAX, R>(act, ctr, Wf, nt0, lane, acc); break;
        case 5: if constexpr (NMAX >= 5) sib_conv_nt<5, NMAX, R>(act, ctr, Wf, nt0, lane, acc); break;
        case 6: if constexpr (NMAX >= 6) sib_conv_nt<6, NMAX, R>(act, ctr, Wf, nt0, lane, acc); break;
        case 7: if constexpr (NMAX >= 7) sib_conv_nt<7, NMAX, R>(act, ctr, Wf, nt0, lane, acc); break;
        case 8: if constexpr (NMAX >= 8) sib_conv_nt<8, NMAX, R>(act, ctr, Wf, nt0, lane, acc); break;
        case 9: if constexpr (NMAX >= 9) sib_conv_nt<9, NMAX, R>(act, ctr, Wf, nt0, lane, acc); break;
        case 10: if constexpr (NMAX >= 10) sib_conv_nt<10, NMAX, R>(act, ctr, Wf, nt0, lane, acc); break;
        case 11: if constexpr (NMAX >= 11) sib_conv_nt<11, NMAX, R>(act, ctr, Wf, nt0, lane, acc); break;
        case 12: if constexpr (NMAX >= 12) sib_conv_nt<12, NMAX, R>(act, ctr, Wf, nt0, lane, acc); break;
        default: break;
    }
}

// A node's recomputed squares: plain stores.  (Agent-scope (sc1) stores, which do
// not keep their lines in the XCD's L2, cut HBM-side fetches 220 -> 194 GB per launch
// but were 2.6 % slower.)
__device__ __forceinline__ void sq_store(_Float16* p, h4 v) { *(h4*)p = v; }

// conv0's im2col for every unit (16 rows x 32 k fp16 each, the columns tree_node
// stages), all units in parallel, into col (the head-partials area, dead during y1)
template <class UT>
__device__ __forceinline__ void sib_col(_Float16* col, const UT* U, int ng, int tid) {
    for (int e = tid; e < ng * 512; e += NTS) {
        const int g = e >> 9, row = (e >> 5) & 15, k = e & 31;
        const UT& u = U[g];
        const int cr = u.cell / BN, cc = u.cell - (u.cell / BN) * BN;
        const Rows r0w = make_rows(cr, cc, 1);
        _Float16 v = (_Float16)0.f;
        if (row < r0w.n && k < 27) {
            const int pr = r0w.r0 + row / r0w.wr, pc = r0w.c0 + row % r0w.wr;
            const int tap = k / 3, cin = k % 3;
            const int rr = pr + tap / 3 - 1, c2 = pc + tap % 3 - 1;
            if (rr >= 0 && rr < BN && c2 >= 0 && c2 < BN) {
                const int bit = bit_of_board(rr, c2);
                const uint32_t bl = (u.board[bit >> 5] >> (bit & 31)) & 1u, wh = (u.board[8 + (bit >> 5)] >> (bit & 31)) & 1u;
                v = (_Float16)(float)(cin == 0 ? bl : (cin == 1 ? wh : 1u - (bl | wh)));
            }
        }
        col[e] = v;
    }
}

// conv0 + BN + ReLU at the <= 9 positions around each unit's stone, wave np: n-tiles
// 2np, 2np+1; into the unit's X0 window and its x0 square
template <int G>
__device__ __forceinline__ void sib_conv0(char* lds, const _Float16* col, const SibUnit* U, int ng,
                                          const float* __restrict__ W, int np, int mh, int lane) {
    const int li = lane & 15, q = lane >> 4;
    constexpr int WIN = wbytes(P_X0) / 2;  // halves per X0 window
    h8 wh[2], wl[2];
    f32x4 ws[2], wt[2];
#pragma unroll
    for (int n = 0; n < 2; n++) {
        const int nt = 2 * np + n, ch0 = nt * 16 + 4 * q;
        const _Float16* wf = (const _Float16*)(W + F16_C0) + ((size_t)nt * 64 + lane) * 8;
        wh[n] = *(const h8*)wf;
        wl[n] = *(const h8*)(wf + 8 * 64 * 8);
        ws[n] = *(const f32x4*)(W + C0_S + ch0);
        wt[n] = *(const f32x4*)(W + C0_T + ch0);
    }
    h8 a[G];
#pragma unroll
    for (int g = 0; g < G; g++) a[g] = *(const h8*)(col + g * 512 + li * 32 + 8 * q);
#pragma unroll
    for (int g = 0; g < G; g++) {
        if (g >= ng) break;
        if (g % SIB_MH != mh) continue;  // the M halves take alternate nodes
        const SibUnit& u = U[g];
        const int cr = u.cell / BN, cc = u.cell - (u.cell / BN) * BN;
        const Rows r0w = make_rows(cr, cc, 1);
        const bool rowok = li < r0w.n;
        const int pr = rowok ? r0w.r0 + li / r0w.wr : 0, pc = rowok ? r0w.c0 + li % r0w.wr : 0;
        _Float16* xw = (_Float16*)lds + g * WIN;
#pragma unroll
        for (int n = 0; n < 2; n++) {
            const int nt = 2 * np + n;
            const int ch0 = nt * 16 + 4 * q;
            const f32x4 s = ws[n], t = wt[n];
            f32x4 acc = zero4();
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[n], a[g], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[n], a[g], acc, 0, 0, 0);
            if (rowok) {
                h4 hi, lo;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    float y = __builtin_fmaf(acc[r], s[r], t[r]);
                    y = y > 0.f ? y : 0.f;
                    const _Float16 h = (_Float16)y;
                    hi[r] = h;
                    lo[r] = (_Float16)(y - (float)h);
                }
                const int off = Win<3>::off(ch0, (pr - cr + 3) * 7 + (pc - cc + 3));
                *(h4*)(xw + off) = hi;
                *(h4*)(xw + Win<3>::plane() + off) = lo;
                _Float16* d = u.own + PATCH_OFF[0] + ((ch0 >> 3) * 9 + (pr - cr + 1) * 3 + (pc - cc + 1)) * 8 + (ch0 & 7);
                sq_store(d, hi);
                sq_store(d + 16 * 9 * 8, lo);
            }
        }
    }
}

// The rows of a pass: units u0 .. u0+ng-1 in order, each its recomputed square of
// radius ro (clipped, row-major), packed back to back; lane li of tile m takes row
// 16m + li (rows past the end repeat the pass's first row, outputs discarded).
template <int NMAX>
struct SibPos {
    int pr[NMAX], pc[NMAX], g[NMAX], row[NMAX];
    bool valid[NMAX];
};

// (this wave's M half mh of the pass's tiles; returns the wave's tile count)
template <int NMAX, int G>
__device__ __forceinline__ int sib_positions(const SibUnit* U, int ng, int ro, int lane, int mh, SibPos<NMAX>& tp) {
    int start[G + 1], r0[G], c0[G], wr[G];
    start[0] = 0;
#pragma unroll
    for (int g = 0; g < G; g++) {
        Rows q = make_rows(0, 0, 0);
        if (g < ng) q = make_rows(U[g].cell / BN, U[g].cell % BN, ro);
        r0[g] = q.r0;
        c0[g] = q.c0;
        wr[g] = q.wr;
        start[g + 1] = start[g] + (g < ng ? q.n : 0);
    }
    const int total = start[G];
    const int T = (total + 15) >> 4, T0 = (T + SIB_MH - 1) / SIB_MH, t0 = mh * T0;
    const int ntw = T - t0 < T0 ? (T - t0 > 0 ? T - t0 : 0) : T0;
    const int li = lane & 15;
#pragma unroll
    for (int m = 0; m < NMAX; m++) {
        int i = (t0 + m) * 16 + li;
        tp.valid[m] = i < total;
        if (i >= total) i = 0;
        int g = 0;
#pragma unroll
        for (int h = 1; h < G; h++) g += i >= start[h] ? 1 : 0;
        int j = 0, rr = 0, R0 = 0, C0 = 0, WR = 1;
#pragma unroll
        for (int h = 0; h < G; h++)
            if (h == g) {
                j = i - start[h];
                R0 = r0[h];
                C0 = c0[h];
                WR = wr[h];
            }
        rr = (int)(((float)j + 0.5f) / (float)WR);  // exact: j < 121, WR <= 11
        tp.g[m] = g;
        tp.row[m] = j;
        tp.pr[m] = R0 + rr;
        tp.pc[m] = C0 + (j - rr * WR);
    }
    return ntw;
}

// One map layer (LAYER 0 = y1: X0 r3 windows -> y1 r2; 1 = x1: Y1 r4 -> x1 r3, + x0;
// 2 = y2: X1 r5 -> y2 r4) over units [u0, u0 + ng): the k-loop, then the epilogue into
// each node's own square (global)
template <int LAYER, int NMAX, int G, class Mid>
__device__ __forceinline__ void sib_map_layer(char* lds, const SibUnit* U, int ng, const float* __restrict__ W, int np,
                                              int mh, int lane, int32_t* tiles, SibStamp<>& st, int si, Mid&& mid) {
    constexpr int R = LAYER + 3, Wd = 2 * R + 1, P = Wd * Wd, ro = R - 1;
    constexpr int MAPOUT = LAYER + 1, S = 2 * ro + 1, SS = S * S;
    constexpr bool SKIP = LAYER == 1;
    SibPos<NMAX> tp;
    const int nt = sib_positions<NMAX, G>(U, ng, ro, lane, mh, tp);
    if (tiles && np == 0 && lane == 0) atomicAdd(tiles, 9 * nt);  // the executed tile-taps, one count per M half
    int ctr[NMAX];
#pragma unroll
    for (int m = 0; m < NMAX; m++) {
        const int cell = U[tp.g[m]].cell, cr = cell / BN, cc = cell - (cell / BN) * BN;
        ctr[m] = tp.g[m] * 2 * 16 * P + (tp.pr[m] - cr + R) * Wd + (tp.pc[m] - cc + R);
    }
    f32x4 acc[2][NMAX];
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int m = 0; m < NMAX; m++) acc[n][m] = zero4();
    // x1's skip input (x0): every load of the epilogue in flight at once (rows past the
    // pass's end read a valid position and are dropped), issued after the k-loop
    // (before it: -0.5 to -1.3 %), so they have landed when the barrier waits for loads
    h4 skh[2][NMAX], skl[2][NMAX];
    auto skip_loads = [&]() {
#pragma unroll
        for (int m = 0; m < NMAX; m++) {
            const MapLoc L = map_loc<0>(U[tp.g[m]], tp.pr[m], tp.pc[m]);
#pragma unroll
            for (int n = 0; n < 2; n++) {
                const int ch0 = (2 * np + n) * 16 + 4 * (lane >> 4);
                const _Float16* p = L.base + (ch0 >> 3) * L.cs + (ch0 & 7);
                skh[n][m] = *(const h4*)p;
                skl[n][m] = *(const h4*)(p + L.lo);
            }
        }
    };
    if (nt > 0) sib_conv<NMAX, R>((const _Float16*)lds, ctr, nt, (const _Float16*)(W + F16_RES0 + LAYER * F16_STRIDE), 2 * np, lane, acc);
    st(si);
    const float* Rw = W + RES0 + LAYER * RES_STRIDE;
    if (SKIP) skip_loads();
    // each row's destination in its node's square, read from the unit table before
    // any store (the stores go through generic pointers the compiler cannot separate
    // from the table)
    _Float16* dst[NMAX];
#pragma unroll
    for (int m = 0; m < NMAX; m++) {
        const SibUnit& u = U[tp.g[m]];
        const int cr = u.cell / BN, cc = u.cell - (u.cell / BN) * BN;
        dst[m] = u.own + PATCH_OFF[MAPOUT] + ((tp.pr[m] - cr + ro) * S + (tp.pc[m] - cc + ro)) * 8;
    }
    f32x4 es[2], et[2];
#pragma unroll
    for (int n = 0; n < 2; n++) {
        const int ch0 = (2 * np + n) * 16 + 4 * (lane >> 4);
        es[n] = *(const f32x4*)(Rw + RES_S + ch0);
        et[n] = *(const f32x4*)(Rw + RES_T + ch0);
    }
    // every global load of the epilogue is issued; the caller's barrier (which waits
    // for them) and the next pass's window fill go here, so the fill's latency hides
    // behind the epilogue
    mid();
    st(si + 1);
#pragma unroll
    for (int n = 0; n < 2; n++) {
        const int ch0 = (2 * np + n) * 16 + 4 * (lane >> 4);
        const f32x4 s = es[n], t = et[n];
#pragma unroll
        for (int m = 0; m < NMAX; m++) {
            if (m >= nt || !tp.valid[m]) continue;
            h4 hi, lo;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float y = __builtin_fmaf(acc[n][m][r], s[r], t[r]);
                if (SKIP) y += (float)skh[n][m][r] + (float)skl[n][m][r];
                y = y > 0.f ? y : 0.f;
                const _Float16 h = (_Float16)y;
                hi[r] = h;
                lo[r] = (_Float16)(y - (float)h);
            }
            _Float16* d = dst[m] + (ch0 >> 3) * SS * 8 + (ch0 & 7);
            sq_store(d, hi);
            sq_store(d + 16 * SS * 8, lo);
        }
    }
}

// x2 + the 1x1 head convs for one unit (Y2 r6 window at LDS 0): wave np = n-tile pair
// over all the unit's M tiles; the head partial sums in tree_node's per-lane chain
// (n-tile 2np then 2np+1, channels in order) and cross-lane order, to hpart
template <class Mid>
__device__ __forceinline__ void sib_head_layer(char* lds, const SibUnit& u, const float* __restrict__ W, int np,
                                               int mh, int lane, float* __restrict__ hpart, int32_t* tiles,
                                               SibStamp<>& st, int si, Mid&& mid) {
    constexpr int layer = 3, NMAX = sib_tiles(8);
    const int cr = u.cell / BN, cc = u.cell - (u.cell / BN) * BN;
    const Rows rows = make_rows(cr, cc, 5);
    const int T = (rows.n + 15) >> 4, T0 = (T + SIB_MH - 1) / SIB_MH, t0 = mh * T0;
    const int nt = T - t0 < T0 ? (T - t0 > 0 ? T - t0 : 0) : T0;
    TilePos<NMAX> tp;
    tile_positions<NMAX, 6>(rows, t0, lane, tp);
    if (tiles && np == 0 && lane == 0) atomicAdd(tiles, 9 * nt);
    int ctr[NMAX];
    tile_centres<NMAX, Win<6>>(tp, cr, cc, ctr);
    f32x4 acc[2][NMAX];
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int m = 0; m < NMAX; m++) acc[n][m] = zero4();
    // the skip input (x1): every load in flight at once, after the k-loop (issued before
    // it, held 44 registers: -0.5 to -1.3 %)
    h4 skh[2][NMAX], skl[2][NMAX];
    auto skip_loads = [&]() {
#pragma unroll
        for (int m = 0; m < NMAX; m++) {
            const MapLoc L = map_loc<2>(u, tp.pr[m], tp.pc[m]);
#pragma unroll
            for (int n = 0; n < 2; n++) {
                const int ch0 = (2 * np + n) * 16 + 4 * (lane >> 4);
                const _Float16* p = L.base + (ch0 >> 3) * L.cs + (ch0 & 7);
                skh[n][m] = *(const h4*)p;
                skl[n][m] = *(const h4*)(p + L.lo);
            }
        }
    };
    if (nt > 0) sib_conv<NMAX, 6>((const _Float16*)lds, ctr, nt, (const _Float16*)(W + F16_RES0 + layer * F16_STRIDE), 2 * np, lane, acc);
    st(si);
    const float* R = W + RES0 + layer * RES_STRIDE;
    skip_loads();
    f32x4 es[2], et[2], e0[2], e1[2], ev[2];
#pragma unroll
    for (int n = 0; n < 2; n++) {
        const int ch0 = (2 * np + n) * 16 + 4 * (lane >> 4);
        es[n] = *(const f32x4*)(R + RES_S + ch0);
        et[n] = *(const f32x4*)(R + RES_T + ch0);
        e0[n] = *(const f32x4*)(W + P_W + ch0);
        e1[n] = *(const f32x4*)(W + P_W + CH + ch0);
        ev[n] = *(const f32x4*)(W + V_W + ch0);
    }
    mid();  // the caller's barrier + the next pass's fill (see sib_map_layer)
    st(si + 1);
    float s0[NMAX], s1[NMAX], sv[NMAX];
#pragma unroll
    for (int m = 0; m < NMAX; m++) s0[m] = s1[m] = sv[m] = 0.f;
#pragma unroll
    for (int n = 0; n < 2; n++) {
        const f32x4 s = es[n], t = et[n], w0 = e0[n], w1 = e1[n], wv = ev[n];
#pragma unroll
        for (int m = 0; m < NMAX; m++) {
            if (m >= nt) continue;
            const h4 xh = skh[n][m], xl = skl[n][m];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float y = __builtin_fmaf(acc[n][m][r], s[r], t[r]) + ((float)xh[r] + (float)xl[r]);
                y = y > 0.f ? y : 0.f;
                s0[m] = __builtin_fmaf(w0[r], y, s0[m]);
                s1[m] = __builtin_fmaf(w1[r], y, s1[m]);
                sv[m] = __builtin_fmaf(wv[r], y, sv[m]);
            }
        }
    }
#pragma unroll
    for (int m = 0; m < NMAX; m++) {
        if (m >= nt) continue;
        float a = s0[m], c = s1[m], v = sv[m];
        a += __shfl_xor(a, 16);
        c += __shfl_xor(c, 16);
        v += __shfl_xor(v, 16);
        a += __shfl_xor(a, 32);
        c += __shfl_xor(c, 32);
        v += __shfl_xor(v, 32);
        const int i = tp.row[m];
        if (lane < 16 && tp.valid[m]) {
            hpart[(np * 3 + 0) * HP_ROWS + i] = a;
            hpart[(np * 3 + 1) * HP_ROWS + i] = c;
            hpart[(np * 3 + 2) * HP_ROWS + i] = v;
        }
    }
}

constexpr int SIB_REC = (HSTRIDE + NTS - 1) / NTS;  // record entries per thread

// node b's head-conv record: its recomputed radius-5 square from hpart (bias, then the
// 4 pairs' partials in order), the rest copied from its base's record
template <class UT>
__device__ __forceinline__ void sib_record(const UT& u, const float* __restrict__ W, float* __restrict__ hbuf,
                                           const float* __restrict__ hpart, const float (&rec)[SIB_REC], int tid) {
    const int cr = u.cell / BN, cc = u.cell - (u.cell / BN) * BN;
    const Rows r4 = make_rows(cr, cc, 5);
    float* h = hbuf + (size_t)u.leaf * HSTRIDE;
#pragma unroll
    for (int k = 0; k < SIB_REC; k++) {
        const int j = tid + k * NTS;
        if (j >= HSTRIDE) break;
        float v = rec[k];
        int pos = -1, which = 0;
        if (j < POS) {
            pos = j;
        } else if (j < 2 * POS) {
            pos = j - POS;
            which = 1;
        } else if (j >= HV_OFF && j < HV_OFF + POS) {
            pos = j - HV_OFF;
            which = 2;
        }
        if (pos >= 0) {
            const int pr = pos / BN, pc = pos % BN;
            if (pr >= r4.r0 && pr < r4.r0 + r4.n / r4.wr && pc >= r4.c0 && pc < r4.c0 + r4.wr) {
                const int i = (pr - r4.r0) * r4.wr + (pc - r4.c0);
                float acc = which == 0 ? W[P_B] : (which == 1 ? W[P_B + 1] : W[V_B]);
#pragma unroll
                for (int q = 0; q < 4; q++) acc += hpart[(q * 3 + which) * HP_ROWS + i];
                v = acc;
            }
        }
        h[j] = v;
    }
}

// list: the grandchildren (tree_grand_order_kernel), list_count entries.  scratch:
// SIB_G patch-sized areas per workgroup.
__global__ __launch_bounds__(NTS, 1) void pv_sib_kernel(TreeArgs A, _Float16* __restrict__ scratch, int n,
                                                       const int32_t* __restrict__ d_count,
                                                       const int32_t* __restrict__ list,
                                                       const int32_t* __restrict__ list_count) {
    __shared__ __attribute__((aligned(16))) char lds[LDS_S];
    SibUnit* const U0 = (SibUnit*)(lds + SIB_U);
    float* hpart = (float*)(lds + SIB_HP);
    const int count = *list_count;
    // XCD-aware interleave: XCD x = blockIdx % 8 takes a contiguous eighth of the list
    // and its workgroups take its groups of SIB_G nodes in turn, so the CUs of one XCD
    // work on neighbouring nodes -- a few roots at a time, whose maps then stay in
    // that XCD's L2
    const int nx = gridDim.x >= 8 ? 8 : 1;
    const int xcd = blockIdx.x % nx, per = gridDim.x / nx, k = blockIdx.x / nx;
    if (k >= per) return;
    const int xchunk = (count + nx - 1) / nx;
    // the XCD's chunks from its queue head in turn, then the other XCDs' (pv_dg_kernel's
    // scheme: no static share, no tail); thread 0 claims one chunk ahead
    int q = 0, claim = 0;
    if (threadIdx.x == 0) claim = atomicAdd(A.queue + xcd, SIB_G);
    _Float16* myscr = scratch + (size_t)blockIdx.x * SIB_G * PATCH_HALVES;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), np = wave & 3, mh = wave >> 2;
    const float* W = A.W;
    int32_t* tiles = A.tiles ? A.tiles + 1 : nullptr;
    SibStamp<> st;
    // the units of the chunk at pos_ (wave 0, one lane per node)
    auto build = [&](SibUnit* Ud, int pos_, int ng_) {
        if (wave == 0 && lane < ng_) {  // the chunk's nodes
            const int b = list[pos_ + lane];
            SibUnit u;
            const int ci = A.cinfo[b];
            const int o = (ci >> 8) & 0x3fffff;
            u.gm = A.maps + (size_t)o * 4 * PV_MAP_HALVES;
            u.leaf = b;
            u.cell = ci & 0xff;
            u.base = A.meta[b];
            u.own = myscr + (size_t)lane * PATCH_HALVES;
#pragma unroll
            for (int w = 0; w < 16; w++) u.board[w] = A.boards[(size_t)b * 16 + w];
            const int pa = u.base;  // the parent: a root child with a patch slot
            u.pcell = A.cinfo[pa] & 0xff;
            u.par = A.patches + (size_t)A.pslot[pa] * PATCH_HALVES;
            Ud[lane] = u;
        }
    };
    for (;;) {
        __syncthreads();  // the previous chunk's readers of U and the chunk entry are done
        if (threadIdx.x == 0) {
            int pb = count, pe = count;  // (none left: the loop ends)
            for (;;) {
                const int qx = (xcd + q) % nx, xb = qx * xchunk, xe = xb + xchunk < count ? xb + xchunk : count;
                if (xb + claim < xe) {
                    pb = xb + claim, pe = xe;
                    claim = atomicAdd(A.queue + qx, SIB_G);
                    break;
                }
                if (++q == nx) break;
                claim = atomicAdd(A.queue + (xcd + q) % nx, SIB_G);
            }
            ((int*)(lds + SIB_POS))[0] = pb;
            ((int*)(lds + SIB_POS))[1] = pe;
        }
        __syncthreads();
        const int pos = ((const int*)(lds + SIB_POS))[0], xe = ((const int*)(lds + SIB_POS))[1];
        if (pos >= xe) break;
        const int ng = xe - pos < SIB_G ? xe - pos : SIB_G;
        SibUnit* const U = U0;
        build(U, pos, ng);
        __syncthreads();
        st(0);
#ifdef GZ_PVINC_STAMPS
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&gz_pvinc_stamps_n[0], (unsigned long long)ng);
#endif
        // The chunk's passes: y1 over all nodes, x1 in passes of 3, y2 in passes of 2,
        // x2 + heads one node at a time.  After each pass's k-loop, a barrier and then
        // the NEXT pass's window fill (LDS-DMA) run before this pass's epilogue, so the
        // fill's latency hides behind the epilogue's VALU work -- unless the next pass
        // reads squares this pass writes (y1 -> x1; x1 -> y2 / y2 -> x2 over the same
        // nodes in small chunks): that fill waits for the epilogue.  The per-pass asm barriers keep the
        // compiler from hoisting every pass's per-lane addresses out of the loop (they
        // would all stay live, and spill).
        const int nx1 = (ng + 2) / 3, ny2 = (ng + 1) / 2, npass = 1 + nx1 + ny2 + ng;
        auto pass_of = [&](int p, int& L, int& u0, int& g) {
            if (p == 0) {
                L = 0, u0 = 0, g = ng;
            } else if (p <= nx1) {
                L = 1, u0 = 3 * (p - 1), g = ng - u0 < 3 ? ng - u0 : 3;
            } else if (p <= nx1 + ny2) {
                L = 2, u0 = 2 * (p - 1 - nx1), g = ng - u0 < 2 ? ng - u0 : 2;
            } else {
                L = 3, u0 = p - 1 - nx1 - ny2, g = 1;
            }
        };
        auto fill = [&](int L, int u0, int g, int t) {
            if (L == 1) sib_fill<1>(lds, U, u0, g, t);
            else if (L == 2) sib_fill<2>(lds, U, u0, g, t);
            else if (L == 3) sib_fill<3>(lds, U, u0, g, t);
        };
        {
            int t = tid;
            asm volatile("" : "+v"(t));
            sib_fill<0>(lds, U, 0, ng, t);
            sib_col((_Float16*)hpart, U, ng, t);
            __syncthreads();  // drains the fill; conv0 then overwrites the nodes' own x0 squares
            st(1);
            const float* Wp = W;
            asm volatile("" : "+s"(Wp));
            sib_conv0<SIB_G>(lds, (const _Float16*)hpart, U, ng, Wp, np, mh, t & 63);
            __syncthreads();
            st(2);
        }
        bool filled = true;  // this pass's windows are in LDS (y1: above)
        for (int p = 0; p < npass; p++) {
            int L, u0, g, L2 = 0, v0 = 0, g2 = 0;
            pass_of(p, L, u0, g);
            // prefetch the next pass's windows unless they hold squares this pass writes
            // (the next layer over some of the same nodes)
            bool pre = p + 1 < npass;
            if (pre) {
                pass_of(p + 1, L2, v0, g2);
                pre = !(L2 == L + 1 && v0 < u0 + g && u0 < v0 + g2);
            }
            const float* Wp = W;
            int t = tid;
            asm volatile("" : "+s"(Wp), "+v"(t));
            if (!filled) {
                fill(L, u0, g, t);
                __syncthreads();
                st(1);
            }
            filled = pre;
            auto mid = [&]() {
                __syncthreads();  // every wave is past this pass's k-loop: the windows are free
                if (pre) fill(L2, v0, g2, t);
            };
            if (L == 0) {
                sib_map_layer<0, sib_tiles(10), SIB_G>(lds, U, g, Wp, np, mh, t & 63, tiles, st, 3, mid);
            } else if (L == 1) {
                sib_map_layer<1, sib_tiles(10), 3>(lds, U + u0, g, Wp, np, mh, t & 63, tiles, st, 6, mid);
            } else if (L == 2) {
                sib_map_layer<2, sib_tiles(11), 2>(lds, U + u0, g, Wp, np, mh, t & 63, tiles, st, 9, mid);
            } else {
                float rec[SIB_REC];  // the base's record entries of this thread, loaded before the x2 k-loop
#pragma unroll
                for (int k = 0; k < SIB_REC; k++) {
                    const int j = t + k * NTS;
                    rec[k] = j < HSTRIDE ? A.hbuf[(size_t)U[u0].base * HSTRIDE + j] : 0.f;
                }
                sib_head_layer(lds, U[u0], Wp, np, mh, t & 63, hpart, tiles, st, 12, mid);
                __syncthreads();  // hpart complete; the next pass's windows have landed
                st(14);
                sib_record(U[u0], Wp, A.hbuf, hpart, rec, t);
                st(15);
                continue;
            }
            __syncthreads();  // the squares are stored; the next pass's windows have landed
            st(3 * L + 5);
        }
    }
}

// one thread per leaf: roots (meta -1) take the next map slot (ord), others -1;
// no patch slot yet
__global__ void tree_roots_kernel(const int32_t* __restrict__ meta, int n, const int32_t* __restrict__ d_count,
                                  int root_cap, int32_t* __restrict__ ord, int32_t* __restrict__ pslot,
                                  int32_t* __restrict__ ctr) {
    const int count = d_count ? (*d_count < n ? *d_count : n) : n;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    int o = -1;
    if (meta[i] == -1) {
        o = atomicAdd(&ctr[0], 1);
        if (o >= root_cap) o = -1;
    }
    ord[i] = o;
    pslot[i] = -1;
}

// node classes (ord: roots' map slots): a root child = meta m >= 0 with ord[m] >= 0;
// a grandchild = meta m >= 0 whose m is such a root child
// boards i and j differ in exactly one bit (one cell changed).  The tags are the
// caller's claim; a leaf whose board does not differ from its tagged parent by one
// cell simply takes the full forward, so a wrong tag costs time, never results
__device__ inline bool one_cell(const uint32_t* __restrict__ boards, int i, int j) {
    int bits = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) bits += __popc(boards[(size_t)i * 16 + k] ^ boards[(size_t)j * 16 + k]);
    return bits == 1;
}

// leaf i is a child of the mapped root m
__device__ inline bool is_child(const int32_t* ord, const uint32_t* boards, int i, int m, int count) {
    return m >= 0 && m < count && ord[m] >= 0 && one_cell(boards, i, m);
}

// one thread per grandchild: its parent claims a patch slot (first come; -2 while
// being claimed, -3 once the slots are exhausted)
__global__ void tree_patch_kernel(const int32_t* __restrict__ meta, int n, const int32_t* __restrict__ d_count,
                                  const int32_t* __restrict__ ord, const uint32_t* __restrict__ boards, int patch_cap,
                                  int32_t* __restrict__ pslot, int32_t* __restrict__ ctr) {
    const int count = d_count ? (*d_count < n ? *d_count : n) : n;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const int m = meta[i];
    if (m < 0 || m >= count || !is_child(ord, boards, m, meta[m], count) || !one_cell(boards, i, m)) return;
    if (atomicCAS(&pslot[m], -1, -2) == -1) {
        const int s = atomicAdd(&ctr[5], 1);
        pslot[m] = s < patch_cap ? s : -3;
    }
}

// lists: roots with a map slot (full forward + maps), every board that is neither
// a root child nor a grandchild whose parent has a patch (full forward); one atomic
// per wave and list.  Grandchildren are chained per parent (ghead / gnext) for
// tree_grand_order_kernel
__device__ inline void wave_append(bool take, int i, int32_t* ctr, int32_t* list) {
    const uint64_t m = __ballot(take);
    if (!m) return;
    int base = 0;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)m) - 1;
    if (lane == leader) base = atomicAdd(ctr, __popcll(m));
    base = __shfl(base, leader);
    if (take) list[base + __popcll(m & ((1ull << lane) - 1))] = i;
}

// the cell of the one stone where boards a and b (16-word leaf rows) differ
__device__ inline int stone_cell(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b) {
    int cell = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t d = a[k] ^ b[k];
        if (d) {
            const int bit = (k & 7) * 32 + __builtin_ctz(d);
            cell = (bit >> 4) * BN + (bit & 15);
        }
    }
    return cell;
}

__global__ void tree_lists_kernel(const int32_t* __restrict__ meta, int n, const int32_t* __restrict__ d_count,
                                  const int32_t* __restrict__ ord, const int32_t* __restrict__ pslot,
                                  const uint32_t* __restrict__ boards, int32_t* __restrict__ ctr,
                                  int32_t* __restrict__ roots, int32_t* __restrict__ full, int32_t* __restrict__ ghead,
                                  int32_t* __restrict__ gnext, int32_t* __restrict__ cinfo,
                                  int32_t* __restrict__ wcount) {
    const int count = d_count ? (*d_count < n ? *d_count : n) : n;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < count;
    const int m = valid ? meta[i] : -3;
    const bool root = valid && m == -1 && ord[i] >= 0;
    const bool child = valid && is_child(ord, boards, i, m, count);
    const bool gc = valid && !child && m >= 0 && m < count && pslot[m] >= 0 && is_child(ord, boards, m, meta[m], count) &&
                    one_cell(boards, i, m);
    wave_append(root, i, ctr + 1, roots);
    wave_append(valid && !root && !child && !gc, i, ctr + 3, full);
    if (gc) gnext[i] = atomicExch(&ghead[pslot[m]], i);  // per parent, any order
    if (valid) {  // the incremental kernels' per-leaf word: root map slot and stone cell
        int ci = -1;
        if (child || gc) {
            const int o = ord[child ? m : meta[m]];
            ci = (gc ? 1 << 30 : 0) | (o << 8) | stone_cell(boards + (size_t)i * 16, boards + (size_t)m * 16);
        }
        cinfo[i] = ci;
    }
    // root children: counted here, listed in leaf order by tree_children_kernel
    const uint64_t c = __ballot(child);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(ctr + 2, __popcll(c));
    if ((threadIdx.x & 63) == 0 && i < n) wcount[i >> 6] = __popcll(c);  // lane 0: i = 64 w
}

// pv_sib_kernel's work list: the root children in LEAF order (a root's children are
// adjacent leaves, so neighbouring list entries share a root's maps).  wcount[w] =
// root children among leaves [64 w, 64 w + 64) (tree_lists_kernel); one workgroup
// of 1024 threads scans the counts in tiles, then (tree_children_scatter_kernel) each
// group's wave writes its leaves' list entries.  cinfo >= 0 with bit 30 clear marks a
// root child.
__global__ __launch_bounds__(1024) void tree_children_kernel(int n, const int32_t* __restrict__ d_count,
                                                            const int32_t* __restrict__ cinfo,
                                                            int32_t* __restrict__ wcount,
                                                            int32_t* __restrict__ children) {
    __shared__ int wsum[16];
    __shared__ int carry;
    const int count = d_count ? (*d_count < n ? *d_count : n) : n;
    const int nw = (count + 63) >> 6;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) carry = 0;
    __syncthreads();
    // exclusive scan of wcount in place, 1024 entries per tile
    for (int t0 = 0; t0 < nw; t0 += 1024) {
        const int w = t0 + tid;
        const int v = w < nw ? wcount[w] : 0;
        int x = v;
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(x, d);
            if (lane >= d) x += y;
        }
        if (lane == 63) wsum[wv] = x;
        __syncthreads();
        if (tid < 16) {
            int y = wsum[tid];
            for (int d = 1; d < 16; d <<= 1) {
                const int z = __shfl_up(y, d, 16);
                if (tid >= d) y += z;
            }
            wsum[tid] = y;  // inclusive over waves
        }
        __syncthreads();
        const int base = carry + (wv ? wsum[wv - 1] : 0);
        if (w < nw) wcount[w] = base + x - v;
        __syncthreads();
        if (tid == 0) carry += wsum[15];
        __syncthreads();
    }
}

// then one wave per 64-leaf group (the loop of 16 waves over the groups was a chain of
// dependent load latencies, 0.4 ms per forward): the group's children in lane order at its
// scanned offset
__global__ __launch_bounds__(1024) void tree_children_scatter_kernel(int n, const int32_t* __restrict__ d_count,
                                                                    const int32_t* __restrict__ cinfo,
                                                                    const int32_t* __restrict__ wcount,
                                                                    int32_t* __restrict__ children) {
    const int count = d_count ? (*d_count < n ? *d_count : n) : n;
    const int w = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w * 64 >= count) return;
    const int i = w * 64 + lane;
    const int ci = i < count ? cinfo[i] : -1;
    const bool child = ci >= 0 && !(ci & (1 << 30));
    const uint64_t m = __ballot(child);
    if (child) children[wcount[w] + __popcll(m & ((1ull << lane) - 1))] = i;
}

// the grandchild list in PARENT order: one thread per leaf; a parent with a patch
// appends its grandchildren (its ghead / gnext chain), a wave's parents in lane
// order.  A root's children are adjacent leaves, so a root's grandchildren end up
// adjacent in the list (the search reserves them one by one during its sequential
// phase, interleaved with every other game's), and pv_grandchild_kernel's
// XCD-contiguous chunks then keep each root's maps in one L2
__global__ void tree_grand_order_kernel(int n, const int32_t* __restrict__ d_count, const int32_t* __restrict__ pslot,
                                        const int32_t* __restrict__ ghead, const int32_t* __restrict__ gnext,
                                        int32_t* __restrict__ ctr, int32_t* __restrict__ grand) {
    const int count = d_count ? (*d_count < n ? *d_count : n) : n;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int ps = i < count ? pslot[i] : -1;
    const int h = ps >= 0 ? ghead[ps] : -1;
    int k = 0;
    for (int g = h; g >= 0; g = gnext[g]) k++;
    // wave prefix sum of k, one atomic per wave
    const int lane = threadIdx.x & 63;
    int incl = k;
    for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
    }
    const int total = __shfl(incl, 63);
    int base = 0;
    if (lane == 63 && total) base = atomicAdd(ctr + 4, total);
    base = __shfl(base, 63);
    int at = base + incl - k;
    for (int g = h; g >= 0; g = gnext[g]) grand[at++] = g;
}

}  // namespace

extern "C" void gz_internal_set_error(const char* msg);
extern "C" int gz_internal_tree_delta(const float* d_weights, const uint32_t* d_boards, const int32_t* d_meta,
                                      const int32_t* d_pslot, const int32_t* d_cinfo, const _Float16* d_maps,
                                      const float* d_pres, _Float16* d_patches, float* d_hbuf, _Float16* d_scratch,
                                      int32_t* d_tiles, int32_t* d_queue, const int32_t* d_children,
                                      const int32_t* d_nchildren, int grid, void* stream);

// Launches of the incremental forward's own kernels (called by gz_pv_forward_tree in
// gz_pvnet.hip, which runs the full kernel on the root and full lists in between).
extern "C" int gz_internal_tree_classify(const int32_t* d_meta, int32_t n, const int32_t* d_count, int32_t root_cap,
                                         int32_t patch_cap, int32_t* d_ord, int32_t* d_pslot, int32_t* d_ctr,
                                         int32_t* d_roots, int32_t* d_full, int32_t* d_grand, int32_t* d_ghead,
                                         int32_t* d_gnext, const uint32_t* d_boards, int32_t* d_cinfo,
                                         int32_t* d_children, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(d_ctr, 0, 32 * sizeof(int32_t), s) != hipSuccess ||  // (ctr[16..32): the queue heads)
        (patch_cap > 0 && hipMemsetAsync(d_ghead, 0xff, (size_t)patch_cap * sizeof(int32_t), s) != hipSuccess)) {
        gz_internal_set_error("gz_pv_forward_tree: memset");
        return GZ_ERR_HIP;
    }
    const int g = (n + 255) / 256;
    tree_roots_kernel<<<g, 256, 0, s>>>(d_meta, n, d_count, root_cap, d_ord, d_pslot, d_ctr);
    tree_patch_kernel<<<g, 256, 0, s>>>(d_meta, n, d_count, d_ord, d_boards, patch_cap, d_pslot, d_ctr);
    // per-wave child counts: past the list's n entries (d_children has n + n / 64 + 1)
    int32_t* wcount = d_children + n;
    tree_lists_kernel<<<g, 256, 0, s>>>(d_meta, n, d_count, d_ord, d_pslot, d_boards, d_ctr, d_roots, d_full, d_ghead,
                                        d_gnext, d_cinfo, wcount);
    tree_children_kernel<<<1, 1024, 0, s>>>(n, d_count, d_cinfo, wcount, d_children);
    tree_children_scatter_kernel<<<(n + 1023) / 1024, 1024, 0, s>>>(n, d_count, d_cinfo, wcount, d_children);
    tree_grand_order_kernel<<<g, 256, 0, s>>>(n, d_count, d_pslot, d_ghead, d_gnext, d_ctr, d_grand);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gz_internal_set_error((std::string("tree classify: ") + hipGetErrorString(e)).c_str());
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}

// the root children through pv_dg_kernel (gz_pvdg.hip; d_pres: the roots' pre-BN
// accumulators), then the grandchildren through pv_sib_kernel
extern "C" int gz_internal_tree_children(const float* d_weights, const uint32_t* d_boards, const int32_t* d_meta,
                                         const int32_t* d_ord, const int32_t* d_pslot, int32_t n,
                                         const int32_t* d_count, const _Float16* d_maps, _Float16* d_patches,
                                         float* d_hbuf, const int32_t* d_grand, const int32_t* d_ngrand,
                                         const int32_t* d_cinfo, _Float16* d_scratch, int32_t* d_tiles,
                                         const int32_t* d_children, const int32_t* d_nchildren, int grid,
                                         const float* d_pres, int32_t* d_queue, void* stream) {
    TreeArgs A{d_cinfo, d_weights, d_boards, d_meta, d_ord, d_pslot, d_maps, d_patches, d_hbuf, d_tiles, d_queue + 8};
    hipStream_t s = (hipStream_t)stream;
    const int rc = gz_internal_tree_delta(d_weights, d_boards, d_meta, d_pslot, d_cinfo, d_maps, d_pres, d_patches,
                                          d_hbuf, d_scratch, d_tiles, d_queue, d_children, d_nchildren, grid, stream);
    if (rc) return rc;
    pv_sib_kernel<<<grid, NTS, 0, s>>>(A, d_scratch, n, d_count, d_grand, d_ngrand);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gz_internal_set_error((std::string("tree children: ") + hipGetErrorString(e)).c_str());
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}

#ifdef GZ_PVINC_STAMPS
// phase stamps of workgroup 0 (-DGZ_PVINC_STAMPS builds, tools/pvinc_bench.py)
extern "C" int gz_pvinc_stamps_read(unsigned long long* out, int reset) {
    // out[0..15] = ticks per phase of pv_sib_kernel, out[32] = its nodes (out[16..31], out[33]: 0)
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gz_pvinc_stamps), 32 * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out + 32, HIP_SYMBOL(gz_pvinc_stamps_n), 2 * sizeof(unsigned long long)) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[32] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(gz_pvinc_stamps), z, sizeof(z)) != hipSuccess) return -1;
        if (hipMemcpyToSymbol(HIP_SYMBOL(gz_pvinc_stamps_n), z, 2 * sizeof(z[0])) != hipSuccess) return -1;
    }
    return 0;
}
#endif
