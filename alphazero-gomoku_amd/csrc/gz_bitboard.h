// gz_bitboard.h -- 15x15 bit-plane boards, the rollout policy and the RNG streams.
//
// Layout: 8 x uint32 words per colour.  Row r lives in word r>>1, half (r&1)*16,
// bit c (0..14); bit 15 of every row and row 15 are guard bits that are always 0.
// Bit index b = 16*r + c, so ascending bit order == the reference's row-major
// order (gomoku_board.py:201-213) and the k-th set bit is the k-th list element.
//
// Direction shifts: "left" neighbour at distance k in direction d is bit b - k*d
// with d in {1 (row), 16 (column), 17 (diagonal), 15 (anti-diagonal)}.  A run
// chain L_k = AND_{j<=k} (X << j*d) is exact on every real cell without any
// masking as long as X has zero guard bits: the first step that would leave the
// board lands on a guard bit (or falls off the word array).  Only final masks
// are ANDed with the empty set.  Proof sketch in DESIGN.md section 3.
//
// Everything here is GZ_HD (host + device) so the per-lane logic can be unit
// tested on the CPU against the oracle; the HIP kernels include it directly.
#pragma once
#include <stdint.h>

#include <type_traits>

#if defined(__HIPCC__)
#define GZ_HD __host__ __device__ inline
#else
#define GZ_HD static inline
#endif

// keep the scheduler from interleaving independent directions (bounds live registers)
#if defined(__HIP_DEVICE_COMPILE__)
#define GZ_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define GZ_SCHED_FENCE() ((void)0)
#endif

// materialise a value in a VGPR here: stops the compiler from re-associating an
// OR-accumulation across directions (which keeps every partial result live)
#if defined(__HIP_DEVICE_COMPILE__)
#define GZ_PIN(x) asm volatile("" : "+v"(x))
#else
#define GZ_PIN(x) ((void)0)
#endif

#define GZ_N 15
#define GZ_CELLS 225
#define GZ_W 8

namespace gz {

// ---------------------------------------------------------------- RNG (gzero/rng.py)
static constexpr uint64_t GOLDEN = 0x9E3779B97F4A7C15ULL;

GZ_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

GZ_HD uint64_t stream_key(uint64_t seed, int64_t game_id, int32_t ply, int32_t sim) {
    uint64_t k = mix64(seed + GOLDEN);
    k = mix64(k ^ ((uint64_t)game_id * GOLDEN));
    k = mix64(k + ((uint64_t)(uint32_t)ply << 32) + (uint64_t)(uint32_t)sim);
    return k;
}

GZ_HD uint64_t draw(uint64_t key, uint32_t i) { return mix64(key + GOLDEN * (uint64_t)(i + 1)); }

GZ_HD double to_unit(uint64_t x) { return (double)(x >> 11) * (1.0 / 9007199254740992.0); }

GZ_HD uint32_t below(uint64_t x, uint32_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__umul64hi(x, (uint64_t)n);
#else
    return (uint32_t)(((unsigned __int128)x * (uint64_t)n) >> 64);
#endif
}

// ---------------------------------------------------------------- bit helpers
GZ_HD int popc(uint32_t x) { return __builtin_popcount(x); }
GZ_HD int ctz(uint32_t x) { return __builtin_ctz(x); }

GZ_HD int cell_to_bit(int cell) { return (cell / GZ_N) * 16 + (cell % GZ_N); }
GZ_HD int bit_to_cell(int bit) { return (bit >> 4) * GZ_N + (bit & 15); }

struct BB {
    uint32_t w[GZ_W];
};

GZ_HD uint32_t valid_word(int i) { return i == 7 ? 0x00007FFFu : 0x7FFF7FFFu; }

GZ_HD BB bb_zero() {
    BB r;
#pragma unroll
    for (int i = 0; i < GZ_W; i++) r.w[i] = 0;
    return r;
}

GZ_HD BB bb_valid() {
    BB r;
#pragma unroll
    for (int i = 0; i < GZ_W; i++) r.w[i] = valid_word(i);
    return r;
}

// word selected by compare/select (no dynamic register indexing -> no scratch)
GZ_HD uint32_t bb_word(const BB& x, int wi) {
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < GZ_W; i++) w = (i == wi) ? x.w[i] : w;
    return w;
}

GZ_HD bool bb_test(const BB& x, int bit) { return (bb_word(x, bit >> 5) >> (bit & 31)) & 1u; }

GZ_HD int bb_count(const BB& x) {
    int n = 0;
#pragma unroll
    for (int i = 0; i < GZ_W; i++) n += popc(x.w[i]);
    return n;
}

GZ_HD bool bb_any(const BB& x) {
    uint32_t a = 0;
#pragma unroll
    for (int i = 0; i < GZ_W; i++) a |= x.w[i];
    return a != 0;
}

// (hi:lo) >> s for 0 < s < 32 (v_alignbit_b32 on gfx950)
GZ_HD uint32_t funnel(uint32_t hi, uint32_t lo, int s) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, (uint32_t)s);
#else
    return (uint32_t)((((uint64_t)hi << 32) | (uint64_t)lo) >> s);
#endif
}

// compile-time loop over word indices (guarantees register-resident words)
template <int I, int N, typename F>
GZ_HD void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// word I of (X << S): bit b receives bit b - S
template <int S, int I>
GZ_HD uint32_t shl_w(const BB& x) {
    constexpr int q = S >> 5, r = S & 31;
    constexpr int ci = I - q, pi = I - q - 1;
    uint32_t cur = 0, prev = 0;
    if constexpr (ci >= 0 && ci < GZ_W) cur = x.w[ci];
    if constexpr (r == 0) {
        return cur;
    } else {
        if constexpr (pi >= 0 && pi < GZ_W) prev = x.w[pi];
        return funnel(cur, prev, 32 - r);
    }
}

// word I of (X >> S): bit b receives bit b + S
template <int S, int I>
GZ_HD uint32_t shr_w(const BB& x) {
    constexpr int q = S >> 5, r = S & 31;
    constexpr int ci = I + q, ni = I + q + 1;
    uint32_t cur = 0, next = 0;
    if constexpr (ci >= 0 && ci < GZ_W) cur = x.w[ci];
    if constexpr (r == 0) {
        return cur;
    } else {
        if constexpr (ni >= 0 && ni < GZ_W) next = x.w[ni];
        return funnel(next, cur, r);
    }
}

template <int S>
GZ_HD BB shl(const BB& x) {
    BB o;
    static_for<0, GZ_W>([&](auto ic) { o.w[decltype(ic)::value] = shl_w<S, decltype(ic)::value>(x); });
    return o;
}

template <int S>
GZ_HD BB shr(const BB& x) {
    BB o;
    static_for<0, GZ_W>([&](auto ic) { o.w[decltype(ic)::value] = shr_w<S, decltype(ic)::value>(x); });
    return o;
}

GZ_HD BB operator&(const BB& a, const BB& b) {
    BB o;
#pragma unroll
    for (int i = 0; i < GZ_W; i++) o.w[i] = a.w[i] & b.w[i];
    return o;
}
GZ_HD BB operator|(const BB& a, const BB& b) {
    BB o;
#pragma unroll
    for (int i = 0; i < GZ_W; i++) o.w[i] = a.w[i] | b.w[i];
    return o;
}

GZ_HD BB empties(const BB& a, const BB& b) {
    BB o;
#pragma unroll
    for (int i = 0; i < GZ_W; i++) o.w[i] = ~(a.w[i] | b.w[i]) & valid_word(i);
    return o;
}

// Constant masks.  Centre buckets of _select_offensive_move step 5
// (ai_agent.py:339-361): Manhattan distance to (7,7) <= 2, in [3, 4], > 4.
// Opening squares of _opening_move (ai_agent.py:152-163): Chebyshev <= 1, <= 2.
#define GZ_MASK_C2 {{0x00000000u, 0x00000000u, 0x00800000u, 0x03E001C0u, 0x008001C0u, 0x00000000u, 0x00000000u, 0x00000000u}}
#define GZ_MASK_C4 {{0x00000000u, 0x00800000u, 0x036001C0u, 0x0C180630u, 0x03600630u, 0x008001C0u, 0x00000000u, 0x00000000u}}
#define GZ_MASK_CE {{0x7FFF7FFFu, 0x7F7F7FFFu, 0x7C1F7E3Fu, 0x7007780Fu, 0x7C1F780Fu, 0x7F7F7E3Fu, 0x7FFF7FFFu, 0x00007FFFu}}
#define GZ_MASK_K3 {{0x00000000u, 0x00000000u, 0x00000000u, 0x01C001C0u, 0x000001C0u, 0x00000000u, 0x00000000u, 0x00000000u}}
#define GZ_MASK_K5 {{0x00000000u, 0x00000000u, 0x03E00000u, 0x03E003E0u, 0x03E003E0u, 0x00000000u, 0x00000000u, 0x00000000u}}

// ------------------------------------------------------------ threat analysis
struct Threats {
    BB win;       // cells where the player's stone completes >= 5 (not yet masked by empties)
    BB make3;     // cells where the player's stone makes a run >= 3 through it
    bool has3;    // the player already has a run >= 3 somewhere
};

// One direction of the threat analysis, computed word by word so that only a
// handful of shifted words are live at a time.
template <int D>
GZ_HD void threats_dir(const BB& m, Threats& t, uint32_t& h) {
    static_for<0, GZ_W>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t a1 = shl_w<D, i>(m), a2 = shl_w<2 * D, i>(m);
        const uint32_t a3 = shl_w<3 * D, i>(m), a4 = shl_w<4 * D, i>(m);
        const uint32_t b1 = shr_w<D, i>(m), b2 = shr_w<2 * D, i>(m);
        const uint32_t b3 = shr_w<3 * D, i>(m), b4 = shr_w<4 * D, i>(m);
        const uint32_t l2 = a1 & a2, l3 = l2 & a3, l4 = l3 & a4;
        const uint32_t r2 = b1 & b2, r3 = r2 & b3, r4 = r3 & b4;
        t.win.w[i] |= l4 | r4 | (a1 & r3) | (l2 & r2) | (l3 & b1);
        t.make3.w[i] |= l2 | r2 | (a1 & b1);
        h |= m.w[i] & l2;
        GZ_PIN(t.win.w[i]);
        GZ_PIN(t.make3.w[i]);
    });
    GZ_PIN(h);
}

GZ_HD Threats threats(const BB& m) {
    Threats t;
    t.win = bb_zero();
    t.make3 = bb_zero();
    uint32_t h = 0;
    threats_dir<1>(m, t, h);
    GZ_SCHED_FENCE();
    threats_dir<16>(m, t, h);
    GZ_SCHED_FENCE();
    threats_dir<17>(m, t, h);
    GZ_SCHED_FENCE();
    threats_dir<15>(m, t, h);
    GZ_SCHED_FENCE();
    t.has3 = h != 0;
    return t;
}

template <int D>
GZ_HD uint32_t run3_dir(const BB& m) {
    uint32_t h = 0;
    static_for<0, GZ_W>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        h |= m.w[i] & shl_w<D, i>(m) & shl_w<2 * D, i>(m);
    });
    return h;
}

// _evaluate_threat_level(board, p) >= 3 (ai_agent.py:403-430)
GZ_HD bool has_run3(const BB& m) {
    return (run3_dir<1>(m) | run3_dir<16>(m) | run3_dir<17>(m) | run3_dir<15>(m)) != 0;
}

GZ_HD int lowest_bit(const BB& x) {
    int r = -1;
#pragma unroll
    for (int i = GZ_W - 1; i >= 0; i--)
        if (x.w[i]) r = i * 32 + ctz(x.w[i]);
    return r;
}

GZ_HD int highest_bit_below(const BB& x, int bound_bit) {
    // highest set bit with index < bound_bit (bound_bit in [0, 256]); -1 if none
    int r = -1;
#pragma unroll
    for (int i = 0; i < GZ_W; i++) {
        int lo = i * 32;
        uint32_t w = x.w[i];
        if (bound_bit <= lo) w = 0;
        else if (bound_bit < lo + 32) w &= (1u << (bound_bit - lo)) - 1u;
        if (w) r = lo + 31 - __builtin_clz(w);
    }
    return r;
}

// index of the k-th (0-based) set bit in ascending order; x must have > k bits
GZ_HD int select_bit(const BB& x, int k) {
    int rem = k, word = 0, base = 0;
    bool found = false;
#pragma unroll
    for (int i = 0; i < GZ_W; i++) {
        int c = popc(x.w[i]);
        bool here = !found && rem < c;
        word = here ? (int)x.w[i] : word;
        base = here ? i * 32 : base;
        rem = (!found && !here) ? rem - c : rem;
        found = found || here;
    }
    uint32_t w = (uint32_t)word;
    int pos = 0;
#pragma unroll
    for (int s = 16; s >= 1; s >>= 1) {
        uint32_t lowmask = (1u << s) - 1u;
        int c = popc(w & lowmask);
        bool up = rem >= c;
        rem = up ? rem - c : rem;
        w = up ? (w >> s) : w;
        pos += up ? s : 0;
    }
    return base + pos;
}

GZ_HD void bb_set(BB& x, int bit) {
    const int wi = bit >> 5;
    const uint32_t m = 1u << (bit & 31);
#pragma unroll
    for (int i = 0; i < GZ_W; i++) x.w[i] |= (i == wi) ? m : 0u;
}

// ---------------------------------------------------------------- rollout policy
// One move of _select_offensive_move (ai_agent.py:306-361) for the side to move
// whose stones are `me` against `op`.  Returns the bit index; *won set when the
// move completes five (step 1); consumes one draw from (key, *cnt) otherwise.
struct Centre {
    BB c2, c4, ce;
};

GZ_HD Centre centre_buckets() {
    Centre c = {GZ_MASK_C2, GZ_MASK_C4, GZ_MASK_CE};
    return c;
}

GZ_HD int policy_move(const BB& me, const BB& op, const BB& e, const Centre& cb, uint64_t key,
                      uint32_t* cnt, bool* won) {
    Threats t = threats(me);
    BB w = t.win & e;
    *won = false;
    if (bb_any(w)) {  // step 1: first immediate win in row-major order
        *won = true;
        return lowest_bit(w);
    }
    BB s;
    if (has_run3(op) || t.has3) {  // step 3 (all legal) / step 4 with an existing run >= 3
        s = e;
    } else {
        s = t.make3 & e;  // step 4
        if (!bb_any(s)) {  // step 5
            s = cb.c2 & e;
            if (!bb_any(s)) s = cb.c4 & e;
            if (!bb_any(s)) s = cb.ce & e;
        }
    }
    int n = bb_count(s);
    uint64_t x = draw(key, (*cnt)++);
    return select_bit(s, (int)below(x, (uint32_t)n));
}

// Offensive part of _simulate (ai_agent.py:276-285) from a non-terminal position,
// `steps0` plies already played (the planner's).  `mover` is the colour to move
// (1/2), `ai` the root AI.  Returns the terminal value (ai_agent.py:287-304).
struct RolloutResult {
    double value;
    BB black, white;
    int n_moves;
    int over, winner;
};

GZ_HD RolloutResult rollout(BB black, BB white, int n_moves, int mover, int ai, int max_depth,
                            uint64_t key, uint32_t* cnt, int steps0 = 0) {
    Centre cb = centre_buckets();
    BB me = mover == 1 ? black : white;
    BB op = mover == 1 ? white : black;
    int over = 0, winner = 0, steps = steps0;
    while (!over && steps < max_depth) {
        BB e = empties(me, op);
        int ne = bb_count(e);
        if (ne == 0) break;
        bool won;
        int b = policy_move(me, op, e, cb, key, cnt, &won);
        bb_set(me, b);
        n_moves++;
        if (won) {
            over = 1;
            winner = mover;
        } else if (ne == 1 || n_moves >= 200) {
            over = 1;
        }
        BB tmp = me;
        me = op;
        op = tmp;
        mover = 3 - mover;
        steps++;
    }
    RolloutResult r;
    r.black = mover == 1 ? me : op;
    r.white = mover == 1 ? op : me;
    r.n_moves = n_moves;
    r.over = over;
    r.winner = winner;
    r.value = !over ? 0.0 : (winner == ai ? 1.0 : (winner != 0 ? -1.0 : 0.1));
    return r;
}

}  // namespace gz
