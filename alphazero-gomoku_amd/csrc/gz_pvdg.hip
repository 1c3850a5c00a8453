// gz_pvdg.hip -- the root children's policy-value forward as a DELTA of the root's,
// gathered (tree mode "delta"; AlphaZeroGomokuNet, neural_network.py:74-91,132-159,
// evaluated once per node the search creates, ai_agent.py:522-523).
//
// A root child is its root plus one stone at cell m.  At the input of residual layer L
// (y1, x1, y2, x2 = L 0..3) the child's activations differ from the root's only in the
// square of radius L+1 around m, so the child's pre-BN accumulator of layer L is the
// root's plus the convolution of that difference D:
//     B_child(p) = B_root(p) + sum_t W_t * D(p + t),    p within radius L+2 of m.
// The root's full forward dumps z = BN(B_root) [+ skip] per layer (gz_pvnet.hip), so
//     child(p) = relu(z(p) + s * sum_t W_t D(p + t) + D_skip(p)),
// and the next layer's D = child - relu(z).  Outputs stay within the f32 rounding of
// a full forward (tests/test_gpu_pvdelta.py: 2e-5 of the full forward, 1e-4 of the
// reference), not bitwise.
//
// Schedule (K below): two workgroups per CU, each (4 waves, one per SIMD) taking chunks
// of 6 consecutive root children (a root's children are adjacent in the list): y1 over
// the 6 nodes, x1 over 3 + 3, then per node pair y2 over the pair and x2 + the 1x1 heads
// over each node -- 12 passes per 6 nodes, each pass one stream of a layer's 576 KB of
// hi/lo weight fragments for up to 12 16-row tiles.
//
// Gather with tap skipping: a pass's output rows (every on-board position of each
// node's radius-(L+2) square) are MFMA M rows; row p needs tap t only if p + t lies in
// the D square (and on the board) -- a set TY x TX.  The rows are counting-sorted by
// that class, so a 16-row tile's tap set (the union of its rows') is small, and a
// tile runs only its taps: 102 tile-taps per node on real searches (92 for the
// unclipped ideal), against 124 for the exact recomputation of the squares -- the delta
// form's saving without pv_delta_kernel's scatter (an LDS read-add-write of the
// accumulators per tap).  Accumulators stay in registers for the whole pass; the D
// squares of the pass's nodes sit in LDS ([plane][16 cg][position][8], a node's square
// row-major, a zero slot for the taps a row does not need), read per tap at the row's
// position + the tap's offset.
//
// Between layers each node's D squares (x0 r1, y1 r2, x1 r3, y2 r4: the patch layout)
// go to the workgroup's scratch in global memory and come back by LDS-DMA for the
// passes that read them -- except where the next pass is the next layer of the same
// first nodes (y1 -> x1 of nodes 0-2, y2 -> x2 of node 2k): those squares go from the
// epilogue straight into the next pass's LDS image.  A node with grandchildren also
// writes its CHILD values into its patch slot for pv_sib_kernel<true> (gz_pvinc.hip).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "gz_f16conv.h"
#include "gz_pvnet.h"
#include "../../include/gzero.h"

using namespace gzpv;

namespace {

using namespace gzc;

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
__device__ uint4 gz_dg_zero16[1];  // zero source of the LDS-DMA fills

constexpr int NTD = 256;  // 4 waves
#ifndef GZ_DG_NTE
#define GZ_DG_NTE 1
#endif
constexpr int PATCH_HALVES = PV_PATCH_HALVES;
constexpr int PATCH_OFF[4] = {0, 9 * 256, 34 * 256, 83 * 256};  // x0 r1, y1 r2, x1 r3, y2 r4 (halves)
__host__ __device__ constexpr int dg_s(int L) { return 2 * L + 3; }  // D-square width (radius L+1)
__host__ __device__ constexpr int dg_ss(int L) { return dg_s(L) * dg_s(L); }
__host__ __device__ constexpr int dg_so(int L) { return 2 * L + 5; }  // output-square width (radius L+2)

// Schedule: two workgroups per CU (<= 80 KB of LDS and <= 256 registers each), so that
// one workgroup's epilogue, fills and barriers run beside the other's MFMAs.  A
// workgroup takes chunks of 6 consecutive nodes; passes of 6 / 3 / 2 / 1 nodes (y1 / x1 /
// y2 / x2), up to 12 output tiles each.  (One workgroup per CU with chunks of 12 and
// passes of 12 / 6 / 4 / 3 -- 87.5 instead of 102 tile-taps per node, but the serial
// phases exposed -- measured 146 against 126 ms per tree forward.)
__host__ __device__ constexpr int dgk_g(int L) { return L == 0 ? 6 : (L == 1 ? 3 : (L == 2 ? 2 : 1)); }
__host__ __device__ constexpr int dgk_npos(int L) { return (dgk_g(L) * dg_ss(L) + 1 + 15) & ~15; }
struct K {
    static constexpr int C = 6;  // nodes per chunk
    __host__ __device__ static constexpr int g(int L) { return dgk_g(L); }
    static constexpr int NPASS = 1 + C / 3 + C / 2 + C;
    // the pass of layer L that takes node gi: y1, x1 x 2, then per node pair k: y2(2k, 2k+1),
    // x2(2k), x2(2k+1) -- so that node 2k's D(y2) goes from the y2 epilogue straight into
    // the x2 pass's LDS image (layer-major y2 x 3, x2 x 6: 1.8 % slower, profiles/r06/ab.md)
    __host__ __device__ static constexpr int pass_of(int L, int gi) {
        return L == 0 ? 0 : (L == 1 ? 1 + gi / 3 : (L == 2 ? 3 + 3 * (gi / 2) : 4 + 3 * (gi / 2) + (gi & 1)));
    }
    // positions of a pass's LDS image: the nodes' squares back to back, then at least one
    // zero slot (the last), rounded to 16 so that a channel group's plane starts at bank 0
    __host__ __device__ static constexpr int npos(int L) { return dgk_npos(L); }
    static constexpr int MAXNPOS = 112;            // npos(2) = max over the layers (static_assert below)
    static constexpr int NMAX = 12;                // output tiles of a pass at most (y2: 2 x 81 rows in 11)
    static constexpr int ROWS = NMAX * 16;         // row-table entries per pass
    static constexpr int GB = 2;                   // epilogue: tiles per load group
    static constexpr int WPS = 2;                  // workgroups per CU
    static constexpr int NKEY = 36;                // row classes (6 x 6 tap sets)
    // LDS
    static constexpr int IN = 0;                   // D squares [2 planes][16 cg][NPOS][8] halves
    static constexpr int IN_BYTES = 32 * MAXNPOS * 16;
    static constexpr int COL = 32 * dgk_npos(0) * 16;  // conv0's im2col (chunk start), behind the y1 image
    static constexpr int HP = IN + IN_BYTES;       // x2: head partials [g(3) nodes][4 waves][3][121] f32
    static constexpr int HP_BYTES = dgk_g(3) * 4 * 3 * 121 * 4;
    static constexpr int ROWT = HP + HP_BYTES;     // row tables [NPASS][ROWS] u32
    static constexpr int MASK = ROWT + NPASS * ROWS * 4;  // [NPASS][16] u32: tap masks [0, 9), rows [9], tile-taps [10]
    static constexpr int HIST = MASK + NPASS * 16 * 4;    // class counters [NPASS][36] (zero between uses), then starts
    static constexpr int U = HIST + 2 * NPASS * NKEY * 4;  // units
    static constexpr int CST = U + C * 128;        // BN scales of the 4 residual layers [4][128], the 1x1 head
    static constexpr int CST_FLOATS = 4 * 128 + 3 * 128 + 4;  // weights [3][128], the 3 head biases
    static constexpr int POS = CST + CST_FLOATS * 4;  // the chunk's first list entry and its queue's end (int)
    static constexpr int LDS = POS + 16;
};
static_assert(dgk_npos(0) <= K::MAXNPOS && dgk_npos(1) <= K::MAXNPOS && dgk_npos(2) == K::MAXNPOS &&
                  dgk_npos(3) <= K::MAXNPOS, "image");
static_assert(K::LDS * K::WPS <= 160 * 1024, "LDS budget");
static_assert(K::COL + K::C * 1024 <= K::IN_BYTES, "im2col behind the y1 image");
static_assert(dgk_g(0) * dg_so(0) * dg_so(0) <= K::ROWS && dgk_g(1) * dg_so(1) * dg_so(1) <= K::ROWS &&
                  dgk_g(2) * dg_so(2) * dg_so(2) <= K::ROWS && dgk_g(3) * dg_so(3) * dg_so(3) <= K::ROWS, "rows");
static_assert(K::C % 6 == 0 && dgk_g(3) == 1, "passes; one x2 node per pass (the record prefetch)");
static_assert(K::C == 6 && dgk_g(1) == 3 && dgk_g(2) == 2, "pass order (K::pass_of, dg_pass_of): 2 x1 triples, 3 y2 pairs");

// The workgroup's scratch: the D squares that cross passes, each map's squares in a
// region of their own ([2 planes][16 cg][square][8] halves per node), sized by what is
// live at once in the pass order -- x0 r1 of the 6 nodes (to the x1 passes' skip), x1 r3
// of the 6 (to the y2 passes and the x2 skip), and one region shared by y1 r2 of nodes
// 3..5 (the first x1 pass takes nodes 0..2's from LDS; dead after the second x1 pass) and
// y2 r4 of node 2k + 1 (node 2k's goes through LDS; dead after x2(2k + 1), before the next
// pair's y2 writes).  429 positions x 512 B = 215 KiB per workgroup instead of 6 patch
// layouts (504 KiB): less to evict from L2 per chunk.
__host__ __device__ constexpr int scr_sq(int map, int node) {
    return (map == 0 ? 9 * node : (map == 2 ? 54 + 49 * node : (map == 1 ? 348 + (node >= 3 ? 25 * (node - 3) : 0) : 348))) * 256;
}
constexpr int SCR_HALVES = (348 + 81) * 256;
static_assert(348 + 3 * 25 <= 348 + 81 && 54 + 49 * 6 == 348, "scratch regions");

struct DgUnit {
    const _Float16* gm;  // the root's maps x0, y1, x1, y2 (hi / lo)
    const float* pre;    // the root's pre-ReLU values of y1, x1, y2, x2
    _Float16* own;       // the workgroup's scratch: this node's D square of map k at own + sq[k]
    _Float16* patch;     // its patch slot (child values for its grandchildren), or nullptr
    int leaf, base, cell, pad0;
    int sq[4];           // halves offsets of its D squares x0 r1, y1 r2, x1 r3, y2 r4 (scr_sq)
    uint32_t board[16];  // the node's bit-plane board (conv0's input)
};
static_assert(sizeof(DgUnit) == 128, "unit size");

struct DgArgs {
    const int32_t* cinfo;  // per leaf: (root map slot << 8) | stone cell (tree_lists_kernel)
    const float* W;
    const uint32_t* boards;
    const int32_t* meta;
    const int32_t* pslot;
    const _Float16* maps;
    const float* pres;
    _Float16* patches;
    float* hbuf;
    int32_t* tiles;  // += executed tile-taps (one 16-row tile x one tap x 128 x 128)
    int32_t* queue;  // [8] per-XCD chunk heads, zero at the launch
};

__device__ inline int iabs(int x) { return x < 0 ? -x : x; }

// Phase stamps (tools/pvinc_bench.py only): -DGZ_PVDG_STAMPS accumulates s_memtime
// deltas of workgroup 0 / thread 0 per phase (vector atomics); compiled out otherwise.
// Phases: 0 chunk start (units, conv0, rows of y1), 1 rows of the next pass, 2..5 the
// k-loops of y1 / x1 / y2 / x2, 6 the barrier after a k-loop, 7..10 the epilogues,
// 11 store drain + barrier, 12 records, 13 fill + barrier
#ifdef GZ_PVDG_STAMPS
__device__ unsigned long long gz_pvdg_stamps[16];
__device__ unsigned long long gz_pvdg_stamps_n[1];
struct DgStamp {
    unsigned long long t = __builtin_amdgcn_s_memtime();
    __device__ void operator()(int i) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();
            atomicAdd(&gz_pvdg_stamps[i], t_ - t);
            t = t_;
        }
    }
};
#else
struct DgStamp {
    __device__ void operator()(int) {}
};
#endif

// global-memory accesses through the unit table's pointers as global (not flat)
// instructions: flat ones count against lgkmcnt too and would hold the LDS waits
#define GZ_GLB __attribute__((address_space(1)))
#ifdef GZ_DG_CHK
// debug builds (tools only): every global access of the kernel checked against the tree
// workspace's bounds; an access outside is counted and redirected to the workspace start
__device__ unsigned long long gz_dg_chk[16];
__device__ const char* gz_dg_lo;
__device__ const char* gz_dg_hi;
__device__ __forceinline__ const void* dg_chk(const void* p, int code) {
    if ((const char*)p < gz_dg_lo || (const char*)p >= gz_dg_hi) {
        atomicAdd(&gz_dg_chk[code], 1ull);
        return gz_dg_lo;
    }
    return p;
}
#define DG_CHK(p, code) dg_chk((p), (code))
#else
#define DG_CHK(p, code) (p)
#endif
template <class T>
__device__ __forceinline__ T gld(const void* p) {
    return *(const GZ_GLB T*)DG_CHK(p, 0);
}
template <class T>
__device__ __forceinline__ void gst(void* p, const T& v) {
    *(GZ_GLB T*)DG_CHK(p, 1) = v;
}

// ------------------------------------------------------------------ rows of a pass
// row entry: node (4 bits) | dy + RO (4) << 4 | dx + RO (4) << 8 | tap mask (9) << 12 |
// valid << 21; tap bit (ty + 1) * 3 + (tx + 1)
// class rank of a tap set (bit 0: -1, bit 1: 0, bit 2: +1) in the order {-1,0,1},
// {-1,0}, {-1}, {0,1}, {0}, {1}: neighbouring classes share taps
__device__ __forceinline__ int set_rank(int b) {
    return b == 7 ? 0 : (b == 3 ? 1 : (b == 1 ? 2 : (b == 6 ? 3 : (b == 2 ? 4 : 5))));
}

// The row tables of every pass of the chunk (nodes U[0, ng)), counting-sorted by class,
// then per pass and tap the tiles that need it.  Ends with the tables written but NOT
// published (the caller's next barrier does).
__device__ __forceinline__ void dg_rows_all(char* lds, const DgUnit* U, int ng, int tid) {
    uint32_t* hist = (uint32_t*)(lds + K::HIST);  // [NPASS][36] counters, then [NPASS][36] starts
    uint32_t* starts = hist + K::NPASS * K::NKEY;
    uint32_t* rt0 = (uint32_t*)(lds + K::ROWT);
    uint32_t* mk0 = (uint32_t*)(lds + K::MASK);
    // candidates: layer-major, then node, then position of the node's output square
    constexpr int N0 = 25, N1 = 49, N2 = 81, N3 = 121;
    const int o1 = ng * N0, o2 = o1 + ng * N1, o3 = o2 + ng * N2, tot = o3 + ng * N3;
    constexpr int PER = (K::C * (N0 + N1 + N2 + N3) + NTD - 1) / NTD;
    int kk[PER], rank[PER];
    uint32_t ent[PER];
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int c = tid + i * NTD;
        kk[i] = -1;
        rank[i] = 0;
        ent[i] = 0;
        if (c >= tot) continue;
        const int L = c < o1 ? 0 : (c < o2 ? 1 : (c < o3 ? 2 : 3));
        const int SO = 2 * L + 5, RO = L + 2, RIN = L + 1;
        const int cl = c - (L == 0 ? 0 : (L == 1 ? o1 : (L == 2 ? o2 : o3)));
        const int gi = cl / (SO * SO), j = cl - gi * (SO * SO), dy = j / SO - RO, dx = j - (j / SO) * SO - RO;
        const int cell = U[gi].cell, cr = cell / BN, cc = cell - (cell / BN) * BN;
        const int pr = cr + dy, pc = cc + dx;
        if (pr < 0 || pr >= BN || pc < 0 || pc >= BN) continue;
        int ty = 0, tx = 0;
#pragma unroll
        for (int d = -1; d <= 1; d++) {
            const int qy = dy + d, qx = dx + d;
            if (qy >= -RIN && qy <= RIN && cr + qy >= 0 && cr + qy < BN) ty |= 1 << (d + 1);
            if (qx >= -RIN && qx <= RIN && cc + qx >= 0 && cc + qx < BN) tx |= 1 << (d + 1);
        }
        if (!ty || !tx) continue;
        uint32_t m = 0;
#pragma unroll
        for (int a = 0; a < 3; a++)
            if ((ty >> a) & 1) m |= (uint32_t)tx << (3 * a);
        const int gl = L == 0 ? 0 : (L == 1 ? 3 : (L == 2 ? 2 : 1));  // nodes per pass of layer L (g(L))
        const int p = K::pass_of(L, gi), u0 = L == 0 ? 0 : (gi / gl) * gl;
        kk[i] = p * K::NKEY + set_rank(ty) * 6 + set_rank(tx);
        ent[i] = (uint32_t)(gi - u0) | ((uint32_t)(dy + RO) << 4) | ((uint32_t)(dx + RO) << 8) | (m << 12) | (1u << 21);
        rank[i] = (int)atomicAdd(&hist[kk[i]], 1u);
    }
    __syncthreads();
    {  // wave w: the bucket starts of passes w, w + 4, ... (exclusive scans of 36 counters), counters back to 0
        const int w = tid >> 6, ln = tid & 63;
        for (int p = w; p < K::NPASS; p += NTD / 64) {
            const uint32_t v = ln < K::NKEY ? hist[p * K::NKEY + ln] : 0u;
            uint32_t x = v;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d);
                if (ln >= d) x += y;
            }
            if (ln < K::NKEY) {
                starts[p * K::NKEY + ln] = x - v;
                hist[p * K::NKEY + ln] = 0u;
            }
            if (ln == 63) mk0[p * 16 + 9] = x;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; i++)
        if (kk[i] >= 0) rt0[(kk[i] / K::NKEY) * K::ROWS + starts[kk[i]] + rank[i]] = ent[i];
    for (int e = tid; e < K::NPASS * K::ROWS; e += NTD)
        if ((uint32_t)(e % K::ROWS) >= mk0[(e / K::ROWS) * 16 + 9]) rt0[e] = 0u;
    __syncthreads();
    {  // wave w, passes w, w + 4, ...: tile tap sets (union of the tile's rows), then per tap the tiles
        const int w = tid >> 6, ln = tid & 63;
        for (int p = w; p < K::NPASS; p += NTD / 64) {
            const uint32_t* rt = rt0 + p * K::ROWS;
            uint32_t tm = 0;
            if (ln < K::NMAX)
#pragma unroll
                for (int k = 0; k < 16; k++) tm |= (rt[ln * 16 + k] >> 12) & 0x1ffu;
            int exec = 0;
#pragma unroll
            for (int t = 0; t < 9; t++) {
                const uint64_t b = __ballot((tm >> t) & 1u);
                if (ln == 0) mk0[p * 16 + t] = (uint32_t)b;
                exec += __popcll(b);
            }
            if (ln == 0) mk0[p * 16 + 10] = (uint32_t)exec;
        }
    }
}

// ------------------------------------------------------------------ the k-loop
// The pass's residual conv for the wave's n-tiles {nt0, nt0+1} over NT output tiles:
// per tap, per 32-channel k-step (the full kernel's k order and its 3 products:
// w_hi a_hi, w_lo a_hi, w_hi a_lo), the tiles that need the tap.  ri[m]: the lane's row
// of tile m: (D-square index of its position + 32) | tap mask << 16.  Activation
// fragments are read one tile ahead unconditionally (deterministic LDS counters: the
// MFMAs of tile m wait only for its own reads), MFMAs only where the tile needs the tap;
// weight fragments through a 4-deep ring refilled 3 k-steps ahead.
template <int NT, int L>
__device__ __forceinline__ void dg_kloop(const char* lds, const uint32_t (&ri)[K::NMAX], const uint32_t* mk,
                                         const _Float16* __restrict__ Wf, int nt0, int lane,
                                         f32x4 (&acc)[2][K::NMAX]) {
    constexpr int S = dg_s(L), NPOS = K::npos(L), CQ = 4, KS = 9 * CQ;
    constexpr int CQB = 4 * NPOS * 16, PLB = 16 * NPOS * 16, ZIDX = NPOS - 1;
    constexpr int KS_BYTES = 8 * 64 * 8 * 2, LO_BYTES = KS * KS_BYTES, RING = 4;
    const int lb = K::IN + (lane >> 4) * NPOS * 16;
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)Wf, 0, 0x7fffffff, 0x00020000);
    const int wo = (nt0 * 64 + lane) * 16;
    auto wload = [&](int ks, int n, int lo) -> h8 {
        return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, wo, ks * KS_BYTES + n * 1024 + lo * LO_BYTES, 0));
    };
    auto addr = [&](int tap, uint32_t r) -> int {
        const int toff = (tap / 3 - 1) * S + (tap - (tap / 3) * 3 - 1);
        const bool v = (r >> (16 + tap)) & 1u;
        return lb + (v ? (int)(r & 0xffffu) - 32 + toff : ZIDX) * 16;
    };
    // Units of two k-steps (a tap's channels 0-63 or 64-127): per tile 12 MFMAs behind one
    // test of the tile's tap mask (with one k-step per unit the per-tile reads, the test
    // and the waits took a third of the loop).  Weights: a ring of 4 k-steps = 2 units,
    // the next unit's pair loaded at the start of a unit into the pair the previous unit
    // released.  Fragments one tile ahead, read unconditionally (the LDS counter is then
    // the same on every path: a tile's MFMAs wait only for its own reads).
    h8 b[RING][2][2];
#pragma unroll
    for (int c = 0; c < 2; c++)
#pragma unroll
        for (int n = 0; n < 2; n++) {
            b[c][n][0] = wload(c, n, 0);
            b[c][n][1] = wload(c, n, 1);
        }
    f32x4 c[2][NT];
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int m = 0; m < NT; m++) c[n][m] = acc[n][m];
    int ad[NT];
#pragma unroll
    for (int m = 0; m < NT; m++) ad[m] = addr(0, ri[m]);
    h8 fh[2][2], fl[2][2];  // [fragment parity][k-step of the pair]
#pragma unroll
    for (int k2 = 0; k2 < 2; k2++) {
        fh[0][k2] = *(const h8*)(lds + ad[0] + k2 * CQB);
        fl[0][k2] = *(const h8*)(lds + ad[0] + k2 * CQB + PLB);
    }
#pragma unroll 1
    for (int tap = 0; tap < 9; tap++) {
        const uint32_t tm = (uint32_t)__builtin_amdgcn_readfirstlane((int)mk[tap]);
#pragma unroll
        for (int h = 0; h < 2; h++) {
            {  // the next unit's k-steps into the pair the previous unit released (past the end: unused)
                const int ksr = tap * CQ + 2 * h + 2;
                const int kn = ksr < KS ? ksr : ksr - KS;
#pragma unroll
                for (int k2 = 0; k2 < 2; k2++)
#pragma unroll
                    for (int n = 0; n < 2; n++) {
                        b[(2 * h + 2 + k2) & 3][n][0] = wload(kn + k2, n, 0);
                        b[(2 * h + 2 + k2) & 3][n][1] = wload(kn + k2, n, 1);
                    }
            }
#pragma unroll
            for (int m = 0; m < NT; m++) {
                // (NT is even: a unit reads an even number of fragment pairs, so tile m's
                // parity is m & 1 on every tap)
                const int pm = m & 1, pn = (m + 1) & 1;
                // the next tile's pair: tile m + 1, else tile 0 of the next unit (the second
                // half of this tap, or the next tap's first, whose address ad[0] holds)
                int na;
                if (m + 1 < NT) na = ad[m + 1] + 2 * h * CQB;
                else na = h == 0 ? ad[0] + 2 * CQB : ad[0];
#pragma unroll
                for (int k2 = 0; k2 < 2; k2++) {
                    fh[pn][k2] = *(const h8*)(lds + na + k2 * CQB);
                    fl[pn][k2] = *(const h8*)(lds + na + k2 * CQB + PLB);
                }
                if (h == 1) ad[m] = addr(tap + 1, ri[m]);  // tile m is read for this tap: the next tap's address
                if ((tm >> m) & 1u) {
#pragma unroll
                    for (int k2 = 0; k2 < 2; k2++) {
                        const int sl = 2 * h + k2;
                        const h8 ah = fh[pm][k2], al = fl[pm][k2];
#pragma unroll
                        for (int n = 0; n < 2; n++) c[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[sl][n][0], ah, c[n][m], 0, 0, 0);
#pragma unroll
                        for (int n = 0; n < 2; n++) c[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[sl][n][1], ah, c[n][m], 0, 0, 0);
#pragma unroll
                        for (int n = 0; n < 2; n++) c[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[sl][n][0], al, c[n][m], 0, 0, 0);
                    }
                }
            }
        }
    }
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int m = 0; m < NT; m++) acc[n][m] = c[n][m];
}

// ------------------------------------------------------------------ epilogue
struct H4x2 {
    h4 h, l;
};
__device__ __forceinline__ float h2f(const H4x2& x, int r) { return (float)x.h[r] + (float)x.l[r]; }
// v split into hi / lo halves at p (global memory) and p + plane_halves
__device__ __forceinline__ void put_hl(_Float16* p, int plane_halves, const f32x4& v) {
    h4 hi, lo;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const _Float16 h = (_Float16)v[r];
        hi[r] = h;
        lo[r] = (_Float16)(v[r] - (float)h);
    }
    gst<h4>(p, hi);
    gst<h4>(p + plane_halves, lo);
}
// the same into LDS
__device__ __forceinline__ void put_hl_lds(_Float16* p, int plane_halves, const f32x4& v) {
    h4 hi, lo;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const _Float16 h = (_Float16)v[r];
        hi[r] = h;
        lo[r] = (_Float16)(v[r] - (float)h);
    }
    *(h4*)p = hi;
    *(h4*)(p + plane_halves) = lo;
}

// The epilogue of a pass (layer L, nodes U[0, g), row table rt): per row,
//   child = relu(z + s * acc + D_skip),  root = relu(z),  D = child - root
// into the node's D square of map L + 1 (its patch: the child value); x2 reduces the
// child values into the 1x1 heads' partial sums (hpart, per wave) instead.  Rows in
// groups of GB tiles, loads ST - 1 groups ahead.
template <int L>
__device__ __forceinline__ void dg_epilogue(char* lds, const DgUnit* U, const uint32_t* rt, int np, int lane,
                                            const f32x4 (&acc)[2][K::NMAX], int nt, int ldsg) {
    constexpr int RO = L + 2, SO = dg_so(L), SSO = SO * SO;
    constexpr bool SKIP = L == 1 || L == 3;
    constexpr int RS = L == 1 ? 1 : 3, SK = 2 * RS + 1, SSK = SK * SK;
    constexpr int GB = K::GB, NGRP = (K::NMAX + GB - 1) / GB, ST = 2;
    float* hpart = (float*)(lds + K::HP);
    const int q = lane >> 4, li = lane & 15;
    const float* cst = (const float*)(lds + K::CST);  // staged at kernel start
    f32x4 es[2], e0[2], e1[2], ev[2];
#pragma unroll
    for (int n = 0; n < 2; n++) {
        const int ch0 = (2 * np + n) * 16 + 4 * q;
        es[n] = *(const f32x4*)(cst + L * 128 + ch0);
        if (L == 3) {
            e0[n] = *(const f32x4*)(cst + 512 + ch0);
            e1[n] = *(const f32x4*)(cst + 640 + ch0);
            ev[n] = *(const f32x4*)(cst + 768 + ch0);
        }
    }
    f32x4 z[ST][GB][2];
    H4x2 dk[ST][GB][2];
    uint32_t ent[ST][GB];
    auto loads = [&](int grp, int st) {
#pragma unroll
        for (int j = 0; j < GB; j++) {
            const int m = grp * GB + j;
            if (m >= K::NMAX) break;  // (an odd NMAX: the last group's second tile)
            const uint32_t e = rt[m * 16 + li];
            ent[st][j] = e;
            const int gi = e & 15, dy = (int)((e >> 4) & 15) - RO, dx = (int)((e >> 8) & 15) - RO;
            const DgUnit& u = U[gi];
            const int cell = u.cell, cr = cell / BN, cc = cell - (cell / BN) * BN;
            const bool v = (e >> 21) & 1u;
            const int pos = v ? (cr + dy) * BN + (cc + dx) : 0;
            const bool near = SKIP && v && iabs(dy) <= RS && iabs(dx) <= RS;
            const int sidx = near ? (dy + RS) * SK + (dx + RS) : 0;
#pragma unroll
            for (int n = 0; n < 2; n++) {
                const int ch0 = (2 * np + n) * 16 + 4 * q;
                z[st][j][n] = gld<f32x4>(u.pre + L * PV_PRE_FLOATS + pos * CH + ch0);
                if (SKIP) {
                    const _Float16* p = u.own + u.sq[L - 1] + ((ch0 >> 3) * SSK + sidx) * 8 + (ch0 & 7);
                    dk[st][j][n] = H4x2{gld<h4>(p), gld<h4>(p + 16 * SSK * 8)};
                }
            }
        }
    };
#pragma unroll
    for (int grp = 0; grp < ST - 1; grp++)
        if (grp * GB < nt) loads(grp, grp);
#pragma unroll
    for (int grp = 0; grp < NGRP; grp++) {
        if (grp * GB >= nt) break;
        const int st = grp % ST;
        if ((grp + ST - 1) * GB < nt) loads(grp + ST - 1, (grp + ST - 1) % ST);
#pragma unroll
        for (int j = 0; j < GB; j++) {
            const int m = grp * GB + j;
            if (m >= K::NMAX) break;
            const uint32_t e = ent[st][j];
            const bool v = (e >> 21) & 1u;
            const int gi = e & 15, dy = (int)((e >> 4) & 15) - RO, dx = (int)((e >> 8) & 15) - RO;
            const bool near = SKIP && iabs(dy) <= RS && iabs(dx) <= RS;
            const int oidx = (dy + RO) * SO + (dx + RO);
            float s0 = 0.f, s1 = 0.f, sv = 0.f;
#pragma unroll
            for (int n = 0; n < 2; n++) {
                const int ch0 = (2 * np + n) * 16 + 4 * q;
                f32x4 y, d;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const float zr = z[st][j][n][r];
                    float tc = __builtin_fmaf(acc[n][m][r], es[n][r], zr);
                    if (SKIP) tc += near ? h2f(dk[st][j][n], r) : 0.f;
                    tc = tc > 0.f ? tc : 0.f;
                    if (L == 3) {
                        s0 = __builtin_fmaf(e0[n][r], tc, s0);
                        s1 = __builtin_fmaf(e1[n][r], tc, s1);
                        sv = __builtin_fmaf(ev[n][r], tc, sv);
                    } else {
                        y[r] = tc;
                        d[r] = tc - (zr > 0.f ? zr : 0.f);
                    }
                }
                if (L < 3 && v) {
                    const DgUnit& u = U[gi];
                    const int o = PATCH_OFF[L + 1] + ((ch0 >> 3) * SSO + oidx) * 8 + (ch0 & 7);
                    if (gi < ldsg) {  // the next pass's image (dg_fill<L + 1>'s layout)
                        constexpr int NPN = K::npos(L + 1 < 4 ? L + 1 : 3), SSN = SSO;
                        put_hl_lds((_Float16*)(lds + K::IN) + ((ch0 >> 3) * NPN + gi * SSN + oidx) * 8 + (ch0 & 7),
                                   16 * NPN * 8, d);
                    } else {
                        put_hl(u.own + u.sq[L + 1] + ((ch0 >> 3) * SSO + oidx) * 8 + (ch0 & 7), 16 * SSO * 8, d);
                    }
                    if (u.patch) put_hl(u.patch + o, 16 * SSO * 8, y);
                }
            }
            if (L == 3) {
                s0 += __shfl_xor(s0, 16);
                s1 += __shfl_xor(s1, 16);
                sv += __shfl_xor(sv, 16);
                s0 += __shfl_xor(s0, 32);
                s1 += __shfl_xor(s1, 32);
                sv += __shfl_xor(sv, 32);
                if (lane < 16 && v) {
                    float* h = hpart + ((gi * 4 + np) * 3) * 121 + oidx;
                    h[0] = s0;
                    h[121] = s1;
                    h[242] = sv;
                }
            }
        }
    }
}

// a node's head-conv record: the radius-5 square from the partials (bias + the 4
// waves' sums), everything else the root's record (rec: this thread's entries of the
// root's record, dg_record_load)
constexpr int REC_K = (HSTRIDE + NTD - 1) / NTD;
__device__ __forceinline__ void dg_record_load(const DgUnit& u, const float* __restrict__ hbuf, float (&rec)[REC_K],
                                               int tid) {
    const float* src = (const float*)DG_CHK(hbuf + (size_t)u.base * HSTRIDE, 3);
#pragma unroll
    for (int k = 0; k < REC_K; k++) {
        const int j = tid + k * NTD;
        rec[k] = j < HSTRIDE ? src[j] : 0.f;
    }
}
__device__ __forceinline__ void dg_record(const DgUnit& u, int g, const float* bias, float* __restrict__ hbuf,
                                          const float* hpart, const float (&rec)[REC_K], int tid) {
    const int cr = u.cell / BN, cc = u.cell - (u.cell / BN) * BN;
    float* h = (float*)DG_CHK(hbuf + (size_t)u.leaf * HSTRIDE, 4);
#pragma unroll
    for (int k = 0; k < REC_K; k++) {
        const int j = tid + k * NTD;
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
            const int dy = pos / BN - cr, dx = pos % BN - cc;
            if (iabs(dy) <= 5 && iabs(dx) <= 5) {
                const int idx = (dy + 5) * 11 + (dx + 5);
                float a = bias[which];
#pragma unroll
                for (int w = 0; w < 4; w++) a += hpart[((g * 4 + w) * 3 + which) * 121 + idx];
                v = a;
            }
        }
        h[j] = v;
    }
}

// ------------------------------------------------------------------ fills and conv0
// the D squares of map L (L >= 1) of nodes U[0, g) into the pass's LDS image by LDS-DMA:
// a lane works out its position's source (a node's square, or zero past them) once per
// 64-position block, then wave w moves channel-group planes [8w, 8w + 8) of it -- the
// planes land at wave-contiguous LDS addresses
template <int L>
__device__ __forceinline__ void dg_fill(char* lds, const DgUnit* U, int g, int tid) {
    constexpr int SS = dg_ss(L), NPOS = K::npos(L), NB = (NPOS + 63) / 64;
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int blk = 0; blk < NB; blk++) {
        const int idx = blk * 64 + lane;
        const _Float16* src = (const _Float16*)gz_dg_zero16;
        int stride = 0;
        if (idx < g * SS) {
            const int gi = idx / SS, j = idx - gi * SS;
            src = U[gi].own + U[gi].sq[L] + j * 8;
            stride = SS * 8;
        }
        char* dst = lds + K::IN + blk * 64 * 16;
        if (idx < NPOS) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int pc = wave * 8 + k;
                __builtin_amdgcn_global_load_lds((glb_void_t*)DG_CHK(src + pc * stride, 2), (lds_void_t*)(dst + pc * NPOS * 16),
                                                 16, 0, 0);
            }
        }
    }
}

// conv0's im2col for every node of the chunk (16 rows x 32 k each: the <= 9 positions
// of the radius-1 square, clipped, row-major; k = tap * 3 + cin)
__device__ __forceinline__ void dg_col(_Float16* col, const DgUnit* U, int ng, int tid) {
    for (int e = tid; e < ng * 512; e += NTD) {
        const int g = e >> 9, row = (e >> 5) & 15, k = e & 31;
        const DgUnit& u = U[g];
        const int cr = u.cell / BN, cc = u.cell - (u.cell / BN) * BN;
        const int r0 = cr > 0 ? cr - 1 : 0, r1 = cr < BN - 1 ? cr + 1 : BN - 1;
        const int c0 = cc > 0 ? cc - 1 : 0, c1 = cc < BN - 1 ? cc + 1 : BN - 1, wr = c1 - c0 + 1;
        _Float16 v = (_Float16)0.f;
        if (row < (r1 - r0 + 1) * wr && k < 27) {
            const int pr = r0 + row / wr, pc = c0 + row % wr;
            const int tap = k / 3, cin = k % 3;
            const int rr = pr + tap / 3 - 1, c2 = pc + tap % 3 - 1;
            if (rr >= 0 && rr < BN && c2 >= 0 && c2 < BN) {
                const int bit = rr * 16 + c2;
                const uint32_t bl = (u.board[bit >> 5] >> (bit & 31)) & 1u, wh = (u.board[8 + (bit >> 5)] >> (bit & 31)) & 1u;
                v = (_Float16)(float)(cin == 0 ? bl : (cin == 1 ? wh : 1u - (bl | wh)));
            }
        }
        col[e] = v;
    }
}

// conv0 + BN + ReLU at the <= 9 positions around each node's stone, D(x0) = child -
// root into the y1 pass's LDS image and the node's x0 square (its patch: the child value)
__device__ __forceinline__ void dg_conv0(char* lds, const _Float16* col, const DgUnit* U, int ng,
                                         const float* __restrict__ W, int np, int lane) {
    constexpr int NPOS = K::npos(0);
    const int li = lane & 15, q = lane >> 4;
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
    _Float16* in = (_Float16*)(lds + K::IN);
    // every node's root x0 values first (one round of latency for the chunk), then the MFMAs
    h4 rxh[K::C][2], rxl[K::C][2];
#pragma unroll
    for (int g = 0; g < K::C; g++) {
        const DgUnit& u = U[g < ng ? g : 0];
        const int cr = u.cell / BN, cc = u.cell - (u.cell / BN) * BN;
        const int r0 = cr > 0 ? cr - 1 : 0, r1 = cr < BN - 1 ? cr + 1 : BN - 1;
        const int c0 = cc > 0 ? cc - 1 : 0, c1 = cc < BN - 1 ? cc + 1 : BN - 1, wr = c1 - c0 + 1;
        const bool rowok = li < (r1 - r0 + 1) * wr;
        const int pr = rowok ? r0 + li / wr : cr, pc = rowok ? c0 + li % wr : cc, pos = pr * BN + pc;
#pragma unroll
        for (int n = 0; n < 2; n++) {
            const int ch0 = (2 * np + n) * 16 + 4 * q;
            const _Float16* rp = u.gm + ((ch0 >> 3) * 256 + pos) * 8 + (ch0 & 7);
            rxh[g][n] = gld<h4>(rp);
            rxl[g][n] = gld<h4>(rp + PV_MAP_PLANE);
        }
    }
#pragma unroll
    for (int g = 0; g < K::C; g++) {
        if (g >= ng) break;
        const h8 a = *(const h8*)(col + g * 512 + li * 32 + 8 * q);
        const DgUnit& u = U[g];
        const int cr = u.cell / BN, cc = u.cell - (u.cell / BN) * BN;
        const int r0 = cr > 0 ? cr - 1 : 0, r1 = cr < BN - 1 ? cr + 1 : BN - 1;
        const int c0 = cc > 0 ? cc - 1 : 0, c1 = cc < BN - 1 ? cc + 1 : BN - 1, wr = c1 - c0 + 1;
        const bool rowok = li < (r1 - r0 + 1) * wr;
        const int pr = rowok ? r0 + li / wr : cr, pc = rowok ? c0 + li % wr : cc;
        const int idx = (pr - cr + 1) * 3 + (pc - cc + 1);
#pragma unroll
        for (int n = 0; n < 2; n++) {
            const int ch0 = (2 * np + n) * 16 + 4 * q;
            f32x4 acc = zero4();
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[n], a, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[n], a, acc, 0, 0, 0);
            if (rowok) {
                const h4 rh = rxh[g][n], rl = rxl[g][n];  // the root's x0
                f32x4 y, d;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    float t = __builtin_fmaf(acc[r], ws[n][r], wt[n][r]);
                    t = t > 0.f ? t : 0.f;
                    y[r] = t;
                    d[r] = t - ((float)rh[r] + (float)rl[r]);
                }
                put_hl_lds(in + ((ch0 >> 3) * NPOS + g * 9 + idx) * 8 + (ch0 & 7), 16 * NPOS * 8, d);
                const int o = PATCH_OFF[0] + ((ch0 >> 3) * 9 + idx) * 8 + (ch0 & 7);
                put_hl(u.own + u.sq[0] + o, 16 * 9 * 8, d);
                if (u.patch) put_hl(u.patch + o, 16 * 9 * 8, y);
            }
        }
    }
}

// ------------------------------------------------------------------ one pass
// the row VGPRs of the lane for every tile, then the k-loop at the smallest tile-count
// instantiation that covers the pass's tiles
template <int L>
__device__ __forceinline__ void dg_pass(const char* lds, const uint32_t* rt, const uint32_t* mk,
                                        const float* __restrict__ W, int np, int lane, f32x4 (&acc)[2][K::NMAX], int nt) {
    constexpr int RIN = L + 1, RO = L + 2, S = dg_s(L), SS = dg_ss(L);
    const int li = lane & 15;
    uint32_t ri[K::NMAX];
#pragma unroll
    for (int m = 0; m < K::NMAX; m++) {
        const uint32_t e = rt[m * 16 + li];
        const int gi = e & 15, dy = (int)((e >> 4) & 15) - RO, dx = (int)((e >> 8) & 15) - RO;
        const int base = gi * SS + (dy + RIN) * S + (dx + RIN) + 32;
        ri[m] = (e >> 21) & 1u ? ((uint32_t)base & 0xffffu) | (((e >> 12) & 0x1ffu) << 16) : 0u;
    }
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int m = 0; m < K::NMAX; m++) acc[n][m] = zero4();
    const _Float16* Wf = (const _Float16*)(W + F16_RES0 + L * F16_STRIDE);
    // the tile count rounded up to a multiple of 4: the padding tiles (no rows, no taps)
    // still cost their fragment reads
#if GZ_DG_NTE
    // instantiated per even tile count up to the layer's most: a padding tile costs
    // its fragment reads and their wait
    constexpr int MT = (dgk_g(L) * dg_so(L) * dg_so(L) + 15) / 16, MTE = (MT + 1) & ~1;
    static_assert(MTE <= K::NMAX, "tiles");
    const int nte = (nt + 1) & ~1;
    if (nte <= 2)
        dg_kloop<2, L>(lds, ri, mk, Wf, 2 * np, lane, acc);
    else if (nte == 4)
        dg_kloop<4, L>(lds, ri, mk, Wf, 2 * np, lane, acc);
    else if (nte == 6 || MTE <= 6)
        dg_kloop<6 < MTE ? 6 : MTE, L>(lds, ri, mk, Wf, 2 * np, lane, acc);
    else if (nte == 8 || MTE <= 8)
        dg_kloop<8 < MTE ? 8 : MTE, L>(lds, ri, mk, Wf, 2 * np, lane, acc);
    else if (nte == 10 || MTE <= 10)
        dg_kloop<10 < MTE ? 10 : MTE, L>(lds, ri, mk, Wf, 2 * np, lane, acc);
    else
        dg_kloop<MTE, L>(lds, ri, mk, Wf, 2 * np, lane, acc);
#else
    if (nt <= 4)
        dg_kloop<4, L>(lds, ri, mk, Wf, 2 * np, lane, acc);
    else if (nt <= 8)
        dg_kloop<8, L>(lds, ri, mk, Wf, 2 * np, lane, acc);
    else
        dg_kloop<K::NMAX, L>(lds, ri, mk, Wf, 2 * np, lane, acc);
#endif
}

// pass p of a chunk of ng nodes: its layer L, first node u0 and node count g (0: empty)
__device__ __forceinline__ void dg_pass_of(int p, int ng, int& L, int& u0, int& g) {
    if (p < 3) {  // (K::pass_of inverted)
        L = p == 0 ? 0 : 1;
        u0 = p == 0 ? 0 : (p - 1) * 3;
    } else {
        const int k = (p - 3) / 3, r = p - 3 - 3 * k;
        L = r == 0 ? 2 : 3;
        u0 = 2 * k + (r == 2 ? 1 : 0);
    }
    g = ng - u0 < K::g(L) ? ng - u0 : K::g(L);
    if (L == 0) u0 = 0, g = ng;
}

__global__ __launch_bounds__(NTD, K::WPS) void pv_dg_kernel(DgArgs A, _Float16* __restrict__ scratch,
                                                           const int32_t* __restrict__ list,
                                                           const int32_t* __restrict__ list_count) {
    __shared__ __attribute__((aligned(16))) char lds[K::LDS];
    DgUnit* const U = (DgUnit*)(lds + K::U);
    const int count = *list_count;
    // XCD-aware interleave: XCD x = blockIdx % 8 takes a contiguous eighth of the list
    // and its workgroups take its chunks in turn, so one XCD works on a few roots at a
    // time (their maps and pre-ReLU values stay in that XCD's L2)
    const int nx = gridDim.x >= 8 ? 8 : 1;
    const int xcd = blockIdx.x % nx, per = gridDim.x / nx, k = blockIdx.x / nx;
    if (k >= per) return;
    const int xchunk = (count + nx - 1) / nx;
    // The XCD's chunks are taken from its queue head in turn (a workgroup that finishes
    // early takes more: no static share, no tail); once the XCD's eighth is exhausted its
    // workgroups help the other XCDs (q = xcd + 1, ...), so no XCD finishes last alone.
    // Thread 0 holds the claim (queue q, offset), made one chunk ahead so that the
    // atomic's latency is hidden, and publishes each chunk's (first entry, end) in LDS.
    int q = 0, claim = 0;
    if (threadIdx.x == 0) claim = atomicAdd(A.queue + xcd, K::C);
    _Float16* myscr = scratch + (size_t)blockIdx.x * SCR_HALVES;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), np = wave;
    const float* W = A.W;
    for (int i = tid; i < K::NPASS * K::NKEY; i += NTD) ((uint32_t*)(lds + K::HIST))[i] = 0u;
    {  // the epilogues' per-channel constants: BN scales of y1, x1, y2, x2, the 1x1 heads' weights and biases
        float* cst = (float*)(lds + K::CST);
        for (int i = tid; i < K::CST_FLOATS; i += NTD) {
            float v;
            if (i < 512) v = W[RES0 + (i >> 7) * RES_STRIDE + RES_S + (i & 127)];
            else if (i < 768) v = W[P_W + (i - 512)];
            else if (i < 896) v = W[V_W + (i - 768)];
            else v = i == 896 ? W[P_B] : (i == 897 ? W[P_B + 1] : (i == 898 ? W[V_B] : 0.f));
            cst[i] = v;
        }
    }
    DgStamp st;
    for (;;) {
        __syncthreads();  // the previous chunk's readers of U, hpart, the tables and POS are done
        if (threadIdx.x == 0) {
            int pb = count, pe = count;  // (none left: the loop ends)
            for (;;) {
                const int qx = (xcd + q) % nx, xb = qx * xchunk, xe = xb + xchunk < count ? xb + xchunk : count;
                if (xb + claim < xe) {
                    pb = xb + claim, pe = xe;
                    claim = atomicAdd(A.queue + qx, K::C);
                    break;
                }
                if (++q == nx) break;
                claim = atomicAdd(A.queue + (xcd + q) % nx, K::C);
            }
            ((int*)(lds + K::POS))[0] = pb;
            ((int*)(lds + K::POS))[1] = pe;
        }
        __syncthreads();
        const int pos = ((const int*)(lds + K::POS))[0], xe = ((const int*)(lds + K::POS))[1];
        if (pos >= xe) break;
        const int ng = xe - pos < K::C ? xe - pos : K::C;
        if (wave == 0 && lane < ng) {
            const int b = list[pos + lane];
            DgUnit u;
            const int ci = A.cinfo[b];
            const int o = (ci >> 8) & 0x3fffff;
            u.gm = A.maps + (size_t)o * 4 * PV_MAP_HALVES;
            u.pre = A.pres + (size_t)o * 4 * PV_PRE_FLOATS;
            u.own = myscr;
            u.sq[0] = scr_sq(0, lane);
            u.sq[1] = scr_sq(1, lane);
            u.sq[2] = scr_sq(2, lane);
            u.sq[3] = scr_sq(3, lane);
            const int ps = A.pslot[b];
            u.patch = ps >= 0 ? A.patches + (size_t)ps * PATCH_HALVES : nullptr;
            u.leaf = b;
            u.base = A.meta[b];
            u.cell = ci & 0xff;
            u.pad0 = 0;
#pragma unroll
            for (int w = 0; w < 16; w++) u.board[w] = A.boards[(size_t)b * 16 + w];
            U[lane] = u;
        }
        __syncthreads();
        {  // conv0 and D(x0): the y1 pass's image (zero past the nodes' squares); every
           // pass's row table
            int t = tid;
            asm volatile("" : "+v"(t));
            dg_col((_Float16*)(lds + K::COL), U, ng, t);
            constexpr int NPOS0 = K::npos(0);
            const int z0 = ng * 9;
            for (int e = t; e < 32 * (NPOS0 - z0); e += NTD) {
                const int pc = e / (NPOS0 - z0), idx = z0 + e % (NPOS0 - z0);
                *(uint4*)(lds + K::IN + (pc * NPOS0 + idx) * 16) = make_uint4(0u, 0u, 0u, 0u);
            }
            __syncthreads();
            const float* Wp = W;
            asm volatile("" : "+s"(Wp));
            dg_conv0(lds, (const _Float16*)(lds + K::COL), U, ng, Wp, np, t & 63);
            dg_rows_all(lds, U, ng, t);
            __syncthreads();  // the y1 image, the row tables and tap masks
#ifdef GZ_DG_CHK
            // every table entry below its pass's row count names a node of that pass
            for (int e = tid; e < K::NPASS * K::ROWS; e += NTD) {
                const int pp = e / K::ROWS;
                int L_, u0_, g_;
                dg_pass_of(pp, ng, L_, u0_, g_);
                const uint32_t tot = ((const uint32_t*)(lds + K::MASK))[pp * 16 + 9];
                const uint32_t en = ((const uint32_t*)(lds + K::ROWT))[e];
                if ((uint32_t)(e % K::ROWS) < tot && (!((en >> 21) & 1u) || (int)(en & 15) >= g_))
                    atomicAdd(&gz_dg_chk[8], 1ull);
                if ((uint32_t)(e % K::ROWS) >= tot && en != 0u) atomicAdd(&gz_dg_chk[9], 1ull);
            }
            if (tid < K::C && (U[tid].cell < 0 || U[tid].cell >= 225) && tid < ng) atomicAdd(&gz_dg_chk[10], 1ull);
#endif
        }
        st(0);
#ifdef GZ_PVDG_STAMPS
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&gz_pvdg_stamps_n[0], (unsigned long long)ng);
#endif
        for (int p = 0; p < K::NPASS; p++) {
            int L, u0, g;
            dg_pass_of(p, ng, L, u0, g);
            if (g <= 0) continue;
            const uint32_t* rt = (const uint32_t*)(lds + K::ROWT) + p * K::ROWS;
            const uint32_t* mk = (const uint32_t*)(lds + K::MASK) + p * 16;
            const int nrows = (int)mk[9], nt = (nrows + 15) >> 4;
            if (A.tiles && tid == 0) atomicAdd(A.tiles, (int)mk[10]);
            const float* Wp = W;
            int t = tid;
            asm volatile("" : "+s"(Wp), "+v"(t));
#ifdef GZ_DG_CHK
            for (int e = tid; e < K::ROWS; e += NTD) {
                const uint32_t en = rt[e];
                if ((uint32_t)e < (uint32_t)nrows && (!((en >> 21) & 1u) || (int)(en & 15) >= g))
                    atomicAdd(&gz_dg_chk[11 + (L > 1 ? 1 : 0)], 1ull);
            }
#endif
            f32x4 acc[2][K::NMAX];
            if (L == 0) dg_pass<0>(lds, rt, mk, Wp, np, t & 63, acc, nt);
            else if (L == 1) dg_pass<1>(lds, rt, mk, Wp, np, t & 63, acc, nt);
            else if (L == 2) dg_pass<2>(lds, rt, mk, Wp, np, t & 63, acc, nt);
            else dg_pass<3>(lds, rt, mk, Wp, np, t & 63, acc, nt);
            st(2 + L);
            __syncthreads();  // every wave is past the k-loop: the image is free
            st(6);
            // the next non-empty pass (its fill follows the epilogue: issued under it, the
            // epilogue's loads would wait for the fill's LDS-DMA -- measured slower)
            int q = p + 1, L2 = 0, v0 = 0, g2 = 0;
            for (; q < K::NPASS; q++) {
                dg_pass_of(q, ng, L2, v0, g2);
                if (g2 > 0) break;
            }
            const bool more = q < K::NPASS;
            // When the next pass is the next layer of this pass's first nodes (y1 -> x1(0..2),
            // y2(2k, 2k+1) -> x2(2k)), those nodes' D squares go straight into the next
            // pass's LDS image (dg_fill's layout) instead of the scratch: no store, no fill,
            // no drain; the pass's other nodes go through the scratch as before.  (The
            // epilogue's scattered 8-B stores of the D squares are 15 % of the kernel.)
            const int ldsg = more && L2 == L + 1 && v0 == u0 && (L == 0 || L == 2) ? g2 : 0;
            const bool to_lds = ldsg > 0;
            if (L == 0) dg_epilogue<0>(lds, U + u0, rt, np, t & 63, acc, nt, ldsg);
            else if (L == 1) dg_epilogue<1>(lds, U + u0, rt, np, t & 63, acc, nt, 0);
            else if (L == 2) dg_epilogue<2>(lds, U + u0, rt, np, t & 63, acc, nt, ldsg);
            else dg_epilogue<3>(lds, U + u0, rt, np, t & 63, acc, nt, 0);
            if (to_lds) {  // the image's zero slots past the nodes' squares (dg_fill writes them)
                const int NPN = L == 0 ? K::npos(1) : K::npos(3), z0 = ldsg * (L == 0 ? dg_ss(1) : dg_ss(3));
                for (int e = t; e < 32 * (NPN - z0); e += NTD) {
                    const int pc = e / (NPN - z0), idx = z0 + e % (NPN - z0);
                    *(uint4*)(lds + K::IN + (pc * NPN + idx) * 16) = make_uint4(0u, 0u, 0u, 0u);
                }
            }
            st(7 + L);
            // vmcnt counts loads, stores and LDS-DMA together in issue order, so each wait
            // below also waits for every older store.  The next pass's fill reads, by
            // LDS-DMA, squares that older passes stored -- and this pass's only when it is
            // the next layer over some of the same nodes (y1 -> the first x1 pass): then
            // every wave's stores complete before a barrier first.  x2: the barrier
            // publishes hpart for the record.
            const bool reads_mine = more && !to_lds && L2 == L + 1 && v0 < u0 + g && u0 < v0 + g2;
            if (reads_mine) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (reads_mine || L == 3) __syncthreads();
            st(11);
            // the fill goes out first; an x2 pass's record (the root's record loaded, the
            // node's written) follows, its loads in flight with the fill's
            if (more && !to_lds) {
                if (L2 == 1) dg_fill<1>(lds, U + v0, g2, t);
                else if (L2 == 2) dg_fill<2>(lds, U + v0, g2, t);
                else if (L2 == 3) dg_fill<3>(lds, U + v0, g2, t);
            }
            if (L == 3) {  // (the root's record entries loaded here: held across the epilogue they were spilled)
                float rec[REC_K];
                dg_record_load(U[u0], A.hbuf, rec, t);
                dg_record(U[u0], 0, (const float*)(lds + K::CST) + 896, A.hbuf, (const float*)(lds + K::HP), rec, t);
                // every thread stores >= 2 record entries after the fill: all but the 2
                // youngest operations done = the fill landed
                asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            st(12);
            __syncthreads();  // the image has landed (and hpart is free again)
            st(13);
        }
    }
}

}  // namespace

extern "C" void gz_internal_set_error(const char* msg);

// the root children (list, list_count entries) of gz_pv_forward_tree
// through pv_dg_kernel; scratch: 12 patch-sized areas per CU (grid = CUs)
extern "C" int gz_internal_tree_delta(const float* d_weights, const uint32_t* d_boards, const int32_t* d_meta,
                                      const int32_t* d_pslot, const int32_t* d_cinfo, const _Float16* d_maps,
                                      const float* d_pres, _Float16* d_patches, float* d_hbuf, _Float16* d_scratch,
                                      int32_t* d_tiles, int32_t* d_queue, const int32_t* d_children,
                                      const int32_t* d_nchildren, int grid, void* stream) {
    DgArgs A{d_cinfo, d_weights, d_boards, d_meta, d_pslot, d_maps, d_pres, d_patches, d_hbuf, d_tiles, d_queue};
    // K::WPS workgroups per grid entry (CU), K::C patch-sized scratch areas each
    static_assert(K::WPS * SCR_HALVES <= PV_SCRATCH_PATCHES * PATCH_HALVES, "scratch");
#ifdef GZ_PVDG_STAMPS
    // stamp builds: GZ_PVDG_WPS=1 runs one workgroup per CU (the k-loop without a co-resident one)
    static const int wps = std::getenv("GZ_PVDG_WPS") && std::getenv("GZ_PVDG_WPS")[0] == '1' ? 1 : K::WPS;
#else
    constexpr int wps = K::WPS;
#endif
#ifdef GZ_DG_CHK
    {
        const char* lo = (const char*)d_hbuf;
        const char* hi = (const char*)(d_scratch + (size_t)grid * PV_SCRATCH_PATCHES * PATCH_HALVES);
        hipMemcpyToSymbolAsync(HIP_SYMBOL(gz_dg_lo), &lo, sizeof(lo), 0, hipMemcpyHostToDevice, (hipStream_t)stream);
        hipMemcpyToSymbolAsync(HIP_SYMBOL(gz_dg_hi), &hi, sizeof(hi), 0, hipMemcpyHostToDevice, (hipStream_t)stream);
    }
#endif
    pv_dg_kernel<<<grid * wps, NTD, 0, (hipStream_t)stream>>>(A, d_scratch, d_children, d_nchildren);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gz_internal_set_error((std::string("tree delta: ") + hipGetErrorString(e)).c_str());
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}

#ifdef GZ_PVDG_STAMPS
// phase stamps of workgroup 0 (-DGZ_PVDG_STAMPS builds, tools/pvinc_bench.py): out[0..15]
// ticks per phase, out[16] nodes
extern "C" int gz_pvdg_stamps_read(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gz_pvdg_stamps), 16 * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out + 16, HIP_SYMBOL(gz_pvdg_stamps_n), sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(gz_pvdg_stamps), z, sizeof(z)) != hipSuccess) return -1;
        if (hipMemcpyToSymbol(HIP_SYMBOL(gz_pvdg_stamps_n), z, sizeof(z[0])) != hipSuccess) return -1;
    }
    return 0;
}
#endif

#ifdef GZ_DG_CHK
// out-of-workspace global accesses per code (loads, stores, fills, record reads, record writes)
extern "C" int gz_pvdg_chk_read(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gz_dg_chk), 16 * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}
#endif
