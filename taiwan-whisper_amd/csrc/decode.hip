// Greedy decoding with a KV cache (generate_step, run_distillation.py:1580-1584;
// HF generation_whisper.py greedy path; logits processors logits_process.py SuppressTokens /
// SuppressTokensAtBegin).
//
//  * tw_decode_attn: one query row per (batch, head) against Tk cached keys — the decoder's
//    self-attention over its cache (Tk = t + 1) and cross-attention over the encoder frames
//    (Tk = 1500).  HBM-bound: every K and V row is read once, 16 B per lane (8 lanes per
//    128-B head row), scores kept in LDS, exact two-pass softmax (max, then exp / sum / P·V).
//  * tw_greedy_select: per batch row, argmax over the vocabulary of the fp32 view of the
//    logits with suppressed ids masked (bitmask; the begin-suppress set only at the first
//    generated step), finished rows forced to eos (= pad), token written to the id matrix and
//    to the next step's input vector, finished flag updated.  Ties resolve to the lowest id
//    (torch.argmax).
//  * tw_select_sample[_ts]: the same selection with the temperature-fallback extensions of HF
//    generate_with_fallback (generation_whisper.py:970-1090): sampling at temperature T by the
//    Gumbel-max trick over the processed row (argmax of x/T + G, G = -log(-log U), U from a
//    counter-based hash of (seed, row, column, id): distributed as multinomial(softmax(x/T)),
//    not torch's RNG stream), and the running sum of log-softmax(processed row)[chosen] that
//    _retrieve_avg_logprobs computes (scores * T undoes the temperature warper).  T and the
//    seed live in a device control word, so one captured decode graph serves every fallback
//    temperature.
//  * tw_token_logprob: log-softmax of a raw logits row at one id (WhisperNoSpeechDetection).
#include "common.h"
#include "decode_impl.h"

#include <algorithm>
#include <cstdlib>

namespace {

using namespace twd;

// U = loads in flight per lane, K/V streamed with nontemporal loads (round 4, tools/bench_decode_attn.py, same box,
// profiles/r04_uv_decode_attn_ab.log): at the c4 shape (fp16, 512 clips x 20 heads over 1500 frames) U = 4 plain
// 665 us, U = 4 nontemporal 620, U = 2 nontemporal 609 (6.45 TB/s), U = 8 782 (occupancy); at 128 x 20 pairs
// U = 4 nontemporal 168 vs U = 2 190 -- hence U = 2 from DA_BIG pairs.
template <typename E, int U>
__device__ __forceinline__ void decode_attn_pair(const DecP& p) {
  const int b = blockIdx.x / p.H, h = blockIdx.x % p.H;
  int tk = p.Tk + (p.tk_dev ? *p.tk_dev : 0);
  if (tk > DA_MAX_TK) tk = DA_MAX_TK;
  decode_attn_body<E, U, true>(p, b, h, 0, tk, nullptr);
}
template <typename E>
__global__ __launch_bounds__(DA_THREADS) void decode_attn_u4_kernel(DecP p) { decode_attn_pair<E, 4>(p); }
template <typename E>
__global__ __launch_bounds__(DA_THREADS) void decode_attn_u2_kernel(DecP p) { decode_attn_pair<E, 2>(p); }

// split over keys (few (clip, head) pairs: batch-1 long-form): blockIdx.y = chunk of S keys; chunks past
// the effective Tk store an empty partial (m = -inf, l = 0); decode_attn_combine_kernel merges them.
// (Tried, r02: the last-arriving chunk combining in place -- agent-scope release + arrival counter --
// saves the second launch at batch 1 (14.6 -> 13.7 us) but every workgroup's release writes back the
// whole L2: 27 -> 202 us at B = 16, and c5 measured no faster.  Two launches it is.)
template <typename E>
__global__ __launch_bounds__(DA_THREADS) void decode_attn_split_kernel(DecP p, int S, float* ws) {
  const int bh = blockIdx.x, c = blockIdx.y;
  const int b = bh / p.H, h = bh % p.H;
  int tk = p.Tk + (p.tk_dev ? *p.tk_dev : 0);
  if (tk > DA_MAX_TK) tk = DA_MAX_TK;
  float* part = ws + ((int64_t)bh * gridDim.y + c) * 66;
  const int lo = c * S, hi = min(tk, lo + S);
  if (lo >= hi) {
    if (threadIdx.x < 64) part[threadIdx.x] = 0.f;
    if (threadIdx.x == 0) {
      part[64] = -INFINITY;
      part[65] = 0.f;
    }
    return;
  }
  decode_attn_body<E>(p, b, h, lo, hi, part);
}

template <typename E>
__global__ __launch_bounds__(64) void decode_attn_combine_kernel(DecP p, int nchunk, const float* ws) {
  combine_row<E>(p, blockIdx.x, nchunk, ws + (int64_t)blockIdx.x * nchunk * 66);
}

struct SelP {
  const void* logits; int64_t ld;
  int V;
  const uint32_t* suppress;   // V-bit mask (nullable)
  const uint32_t* begin;      // V-bit mask applied when apply_begin (nullable)
  int apply_begin;
  int64_t eos;
  uint8_t* done;
  int64_t* ids; int64_t ld_ids; int col;
  int64_t* next;              // [B] next-step input ids
  const int* t_dev;           // nullable: col = *t_dev + col, begin mask applied when col == begin_col
  int begin_col;
  const uint32_t* ctl;        // nullable: per row b, ctl[3b] = bits of 1/T (0: greedy), ctl[3b+1], [3b+2] = seed lo, hi
  float* sum_logp;            // nullable: += log-prob of the chosen token while the row is live
  int vec;                    // rows 16-B aligned and padded to a multiple of 8 ids: 16-B loads
};

// f(v, x, suppressed, begin_suppressed) over this thread's ids of a logits row: chunks of 8
// consecutive ids (one 16-B load, one word of each mask), chunk c = tid, tid + 256, ...
template <typename E, class F>
__device__ __forceinline__ void for_row(const SelP& p, const E* row, F&& f, int lo = 0, int hi = -1) {
  if (hi < 0) hi = p.V;                                  // [lo, hi), lo a multiple of 8
  for (int v0 = lo + (int)threadIdx.x * 8; v0 < hi; v0 += 256 * 8) {
    float xs[8];
    if (p.vec) {
      load8(row + v0, xs);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) xs[j] = v0 + j < p.V ? to_f32(row[v0 + j]) : -INFINITY;
    }
    const uint32_t ws = p.suppress ? p.suppress[v0 >> 5] >> (v0 & 31) : 0u;   // 8 ids never straddle a word
    const uint32_t wb = p.begin ? p.begin[v0 >> 5] >> (v0 & 31) : 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (v0 + j < hi) f(v0 + j, xs[j], ((ws >> j) & 1u) != 0u, ((wb >> j) & 1u) != 0u);
  }
}

// (max, sum exp(x - max)) pairs: running logsumexp
__device__ __forceinline__ void lse_add(float& m, float& s, float x) {
  if (x > m) { s = s * __expf(m - x) + 1.f; m = x; }
  else s += __expf(x - m);
}
__device__ __forceinline__ void lse_merge(float& m, float& s, float om, float os) {
  const float mx = fmaxf(m, om);
  s = (mx == -INFINITY) ? 0.f : s * __expf(m - mx) + os * __expf(om - mx);
  m = mx;
}
__device__ __forceinline__ float lse_val(float m, float s) { return m == -INFINITY ? -INFINITY : m + __logf(s); }

// Gumbel(0,1) noise of token v at (row b, column col): splitmix64 of a distinct 64-bit key
// (b, col, v < 2^21 each) -> 24-bit uniform in (0, 1)
__device__ __forceinline__ float gumbel(uint64_t seed, int b, int col, int v) {
  uint64_t x = seed + 0x9E3779B97F4A7C15ull *
                          ((((uint64_t)(uint32_t)b) << 42) ^ (((uint64_t)(uint32_t)col) << 21) ^ (uint64_t)(uint32_t)v);
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  const float u = ((float)(x >> 40) + 0.5f) * (1.0f / 16777216.0f);
  return -__logf(-__logf(u));
}

// row b's sampling control: its own temperature and seed, so the rows of one batch can be independent fallback
// attempts (each row's draw keyed by (its seed, column, id) only: a row decodes the same tokens whatever batch
// it runs in)
__device__ __forceinline__ void read_ctl(const uint32_t* ctl, int b, float& inv_t, uint64_t& seed) {
  inv_t = ctl ? __uint_as_float(ctl[3 * b]) : 0.f;
  seed = ctl ? ((uint64_t)ctl[3 * b + 2] << 32 | ctl[3 * b + 1]) : 0ull;
}

// block (256 threads) argmax with lowest-id ties, result broadcast to thread 0's registers
__device__ __forceinline__ void block_argmax(float& v, int& i, float (*sv)[4], int (*si)[4], int slot) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(i, o, 64);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
  if (lane == 0) { sv[slot][wave] = v; si[slot][wave] = i; }
  __syncthreads();
  if (tid == 0)
    for (int w = 1; w < 4; ++w)
      if (sv[slot][w] > v || (sv[slot][w] == v && si[slot][w] < i)) { v = sv[slot][w]; i = si[slot][w]; }
}
__device__ __forceinline__ void block_lse(float& m, float& s, float (*sv)[4], int slot) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lse_merge(m, s, __shfl_xor(m, o, 64), __shfl_xor(s, o, 64));
  if (lane == 0) { sv[slot][wave] = m; sv[slot + 1][wave] = s; }
  __syncthreads();
  if (tid == 0)
    for (int w = 1; w < 4; ++w) lse_merge(m, s, sv[slot][w], sv[slot + 1][w]);
}

__device__ __forceinline__ bool bit(const uint32_t* m, int v) { return m && ((m[v >> 5] >> (v & 31)) & 1u); }

// Selection over a row is split into scan (per-thread accumulation over a slice of the vocabulary),
// block reduction, and finish (thread 0: merge, pick, bookkeeping).  Few rows (batch-1 long-form): the
// row is cut into G slices, one workgroup each, partials to the per-device scratch block, and a second
// kernel merges them in slice order and finishes -- one 256-thread workgroup per row scanning 51 865
// logits took ~78 us per step; many rows: one workgroup per row does all three.
struct GreedyAcc {
  float best, sbest, m, se;
  int besti, sbesti;
};
constexpr int SEL_WORDS = 8;     // words per partial in the scratch block

__device__ __forceinline__ void greedy_init(GreedyAcc& a) {
  a.best = a.sbest = a.m = -INFINITY;
  a.se = 0.f;
  a.besti = a.sbesti = 0x7fffffff;
}
__device__ __forceinline__ void greedy_merge(GreedyAcc& a, const GreedyAcc& o, bool sample, bool lse) {
  if (o.best > a.best || (o.best == a.best && o.besti < a.besti)) { a.best = o.best; a.besti = o.besti; }
  if (sample && (o.sbest > a.sbest || (o.sbest == a.sbest && o.sbesti < a.sbesti))) { a.sbest = o.sbest; a.sbesti = o.sbesti; }
  if (lse) lse_merge(a.m, a.se, o.m, o.se);
}
template <typename E>
__device__ __forceinline__ void greedy_scan(const SelP& p, const E* row, int b, bool sample, float inv_t, uint64_t seed,
                                            GreedyAcc& a, int lo, int hi) {
  const bool lse = p.sum_logp != nullptr;
  for_row(p, row, [&](int v, float x, bool sup, bool beg) {
    if (sup || (p.apply_begin && beg)) x = -INFINITY;
    if (x > a.best || (x == a.best && v < a.besti)) { a.best = x; a.besti = v; }
    if (x > -INFINITY) {
      if (lse) lse_add(a.m, a.se, x);
      if (sample) {
        const float g = x * inv_t + gumbel(seed, 0, p.col, v);
        if (g > a.sbest || (g == a.sbest && v < a.sbesti)) { a.sbest = g; a.sbesti = v; }
      }
    }
  }, lo, hi);
}
// block reduction: the result in thread 0's a
__device__ __forceinline__ void greedy_block(GreedyAcc& a, bool sample, bool lse, float (*sv)[4], int (*si)[4]) {
  block_argmax(a.best, a.besti, sv, si, 0);
  if (sample) block_argmax(a.sbest, a.sbesti, sv, si, 1);
  if (lse) block_lse(a.m, a.se, sv, 2);
}
template <typename E>
__device__ __forceinline__ void greedy_finish(const SelP& p, const E* row, int b, const GreedyAcc& a, bool sample) {
  int pick = sample ? a.sbesti : a.besti;
  if (pick == 0x7fffffff) pick = 0;              // every logit masked / NaN: id 0 (torch argmax of all -inf)
  const bool fin = p.done[b] != 0;
  const int64_t tok = fin ? p.eos : (int64_t)pick;
  p.ids[b * p.ld_ids + p.col] = tok;
  p.next[b] = tok;
  p.done[b] = (fin || tok == p.eos) ? 1 : 0;
  if (p.sum_logp && !fin) p.sum_logp[b] += to_f32(row[pick]) - lse_val(a.m, a.se);
}
__device__ __forceinline__ void sel_prologue(SelP& p) {
  if (p.t_dev) {
    p.col += *p.t_dev;
    p.apply_begin = p.col == p.begin_col;
  }
}

// grid (G, B): G == 1 -> scan the whole row and finish; G > 1 -> partial of slice blockIdx.x into ws
template <typename E>
__global__ __launch_bounds__(256) void greedy_select_kernel(SelP p, int slice, float* ws) {
  __shared__ float sv[4][4];
  __shared__ int si[4][4];
  const int g = blockIdx.x, G = gridDim.x, b = blockIdx.y, tid = threadIdx.x;
  sel_prologue(p);
  float inv_t;
  uint64_t seed;
  read_ctl(p.ctl, b, inv_t, seed);
  const bool sample = inv_t > 0.f, lse = p.sum_logp != nullptr;
  const E* row = (const E*)p.logits + b * p.ld;
  GreedyAcc a;
  greedy_init(a);
  const int lo = G == 1 ? 0 : g * slice, hi = G == 1 ? p.V : min(p.V, lo + slice);
  greedy_scan(p, row, b, sample, inv_t, seed, a, lo, hi);
  greedy_block(a, sample, lse, sv, si);
  if (tid != 0) return;
  if (G == 1) {
    greedy_finish(p, row, b, a, sample);
  } else {
    float* w = ws + ((int64_t)b * G + g) * SEL_WORDS;
    w[0] = a.best; w[1] = a.sbest; w[2] = a.m; w[3] = a.se;
    w[4] = __int_as_float(a.besti); w[5] = __int_as_float(a.sbesti);
  }
}

template <typename E>
__global__ __launch_bounds__(64) void greedy_merge_kernel(SelP p, int G, const float* ws) {
  const int b = blockIdx.x;
  if (threadIdx.x != 0) return;
  sel_prologue(p);
  float inv_t;
  uint64_t seed;
  read_ctl(p.ctl, b, inv_t, seed);
  const bool sample = inv_t > 0.f, lse = p.sum_logp != nullptr;
  GreedyAcc a;
  greedy_init(a);
  for (int g = 0; g < G; ++g) {
    const float* w = ws + ((int64_t)b * G + g) * SEL_WORDS;
    GreedyAcc o;
    o.best = w[0]; o.sbest = w[1]; o.m = w[2]; o.se = w[3];
    o.besti = __float_as_int(w[4]); o.sbesti = __float_as_int(w[5]);
    greedy_merge(a, o, sample, lse);
  }
  greedy_finish(p, (const E*)p.logits + b * p.ld, b, a, sample);
}


// Timestamp decoding (HF WhisperTimeStampLogitsProcessor, applied after the suppress processors):
// <|notimestamps|> masked; timestamps in pairs (after ts,ts -> text; after text,ts -> ts or eos);
// timestamps non-decreasing (none below the last one, or below last+1 unless closing a pair);
// at the window's first step only timestamps <= ts_begin + max_initial; and when the probability
// mass of all timestamps exceeds the best text token (logsumexp over timestamps > max text logit,
// the log_softmax shift cancels) only timestamps are eligible.  One pass per row gathers the
// text argmax, the timestamp argmax and the timestamp logsumexp; last_ts[b] keeps the row's last
// emitted timestamp (-1: none in this window).
struct SelTsP {
  SelP s;
  int begin_col;              // first generated column of the window
  int ts_begin, no_ts, max_initial;
  int* last_ts;
};

struct TsAcc {
  float bt, bs, se, tm, tse;      // best text, best timestamp, sum exp(ts - bs), text logsumexp (m, s)
  int it, is;
};
__device__ __forceinline__ void ts_init(TsAcc& a) {
  a.bt = a.bs = a.tm = -INFINITY;
  a.se = a.tse = 0.f;
  a.it = a.is = 0x7fffffff;
}
__device__ __forceinline__ void ts_merge(TsAcc& a, const TsAcc& o, bool lse) {
  if (o.bt > a.bt || (o.bt == a.bt && o.it < a.it)) { a.bt = o.bt; a.it = o.it; }
  const float mx = fmaxf(a.bs, o.bs);
  const float ns = (mx == -INFINITY) ? 0.f : a.se * __expf(a.bs - mx) + o.se * __expf(o.bs - mx);
  if (o.bs > a.bs || (o.bs == a.bs && o.is < a.is)) a.is = o.is;
  a.bs = mx;
  a.se = ns;
  if (lse) lse_merge(a.tm, a.tse, o.tm, o.tse);
}
// the row's timestamp-rule state at column p.col
struct TsRow {
  bool first, last_ts, pen_ts;
  int lim, ts_hi;
};
__device__ __forceinline__ TsRow ts_row(const SelTsP& q, int b) {
  const SelP& p = q.s;
  TsRow r;
  r.first = p.col == q.begin_col;
  const int64_t* idr = p.ids + b * p.ld_ids;
  const bool has1 = p.col - 1 >= q.begin_col, has2 = p.col - 2 >= q.begin_col;
  r.last_ts = has1 && idr[p.col - 1] >= q.ts_begin;
  r.pen_ts = !has2 || idr[p.col - 2] >= q.ts_begin;
  const int lt = q.last_ts[b];
  r.lim = lt < 0 ? q.ts_begin : ((r.last_ts && !r.pen_ts) ? lt : lt + 1);
  r.ts_hi = (r.first && q.max_initial >= 0) ? q.ts_begin + q.max_initial : 0x7fffffff;
  return r;
}
// eligibility of id v before the "timestamp mass wins" rule
__device__ __forceinline__ bool ts_masked(const SelTsP& q, const TsRow& r, int v, bool sup, bool beg) {
  bool m = sup || (r.first && beg) || v == q.no_ts;
  if (v >= q.ts_begin) {
    if (r.last_ts && r.pen_ts) m = true;
    if (v < r.lim || v > r.ts_hi) m = true;
  } else if ((r.last_ts && !r.pen_ts && v < q.s.eos) || r.first) {
    m = true;
  }
  return m;
}
template <typename E>
__device__ __forceinline__ void ts_scan(const SelTsP& q, const TsRow& r, const E* row, TsAcc& a, int lo, int hi) {
  const bool lse = q.s.sum_logp != nullptr;
  for_row(q.s, row, [&](int v, float x, bool sup, bool beg) {
    if (ts_masked(q, r, v, sup, beg) || !(x > -INFINITY)) return;
    if (v >= q.ts_begin) {
      if (x > a.bs) { a.se = a.se * __expf(a.bs - x) + 1.f; a.bs = x; a.is = v; }
      else { a.se += __expf(x - a.bs); if (x == a.bs && v < a.is) a.is = v; }
    } else {
      if (x > a.bt || (x == a.bt && v < a.it)) { a.bt = x; a.it = v; }
      if (lse) lse_add(a.tm, a.tse, x);
    }
  }, lo, hi);
}
// block reduction (waves by shuffles, then thread 0 over the 4 waves): the result in thread 0's a
__device__ __forceinline__ void ts_block(TsAcc& a, bool lse, float (*sv)[8], int (*si)[2]) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    TsAcc x;
    x.bt = __shfl_xor(a.bt, o, 64); x.bs = __shfl_xor(a.bs, o, 64); x.se = __shfl_xor(a.se, o, 64);
    x.tm = __shfl_xor(a.tm, o, 64); x.tse = __shfl_xor(a.tse, o, 64);
    x.it = __shfl_xor(a.it, o, 64); x.is = __shfl_xor(a.is, o, 64);
    ts_merge(a, x, lse);
  }
  if (lane == 0) {
    sv[wave][0] = a.bt; sv[wave][1] = a.bs; sv[wave][2] = a.se; sv[wave][3] = a.tm; sv[wave][4] = a.tse;
    si[wave][0] = a.it; si[wave][1] = a.is;
  }
  __syncthreads();
  if (tid == 0)
    for (int w = 1; w < 4; ++w) {
      TsAcc x;
      x.bt = sv[w][0]; x.bs = sv[w][1]; x.se = sv[w][2]; x.tm = sv[w][3]; x.tse = sv[w][4];
      x.it = si[w][0]; x.is = si[w][1];
      ts_merge(a, x, lse);
    }
}
// finish (whole workgroup; the merged accumulator in thread 0's a): the timestamp-mass rule, the
// temperature-sampling pass over the processed row (Gumbel-max) when T > 0, the pick and bookkeeping
template <typename E>
__device__ __forceinline__ void ts_finish(const SelTsP& q, const TsRow& r, int b, TsAcc& a, float (*sx)[4],
                                          int (*sxi)[4]) {
  __shared__ int s_mask_text;
  const SelP& p = q.s;
  const int tid = threadIdx.x;
  float inv_t;
  uint64_t seed;
  read_ctl(p.ctl, b, inv_t, seed);
  const bool sample = inv_t > 0.f;
  const E* row = (const E*)p.logits + b * p.ld;
  if (tid == 0) {
    const float ts_lse = a.bs == -INFINITY ? -INFINITY : a.bs + __logf(a.se);
    s_mask_text = (a.bs > -INFINITY && ts_lse > a.bt) ? 1 : 0;   // timestamp mass wins: text masked
  }
  __syncthreads();
  const bool mask_text = s_mask_text != 0;
  int spick = 0x7fffffff;
  if (sample) {                                          // second pass: Gumbel-max over the processed row
    float sb = -INFINITY;
    for_row(p, row, [&](int v, float x, bool sup, bool beg) {
      if (ts_masked(q, r, v, sup, beg) || !(x > -INFINITY) || (mask_text && v < q.ts_begin)) return;
      const float g = x * inv_t + gumbel(seed, 0, p.col, v);
      if (g > sb || (g == sb && v < spick)) { sb = g; spick = v; }
    });
    block_argmax(sb, spick, sx, sxi, 2);
  }
  if (tid == 0) {
    const float ts_l = lse_val(a.bs, a.se);
    int best;
    if (mask_text) best = a.is;
    else if (a.bt >= a.bs && a.it != 0x7fffffff) best = a.it;       // text ids < timestamp ids: ties -> text
    else if (a.is != 0x7fffffff) best = a.is;
    else best = 0;
    if (sample) best = spick == 0x7fffffff ? best : spick;
    const bool fin = p.done[b] != 0;
    const int64_t tok = fin ? p.eos : (int64_t)best;
    p.ids[b * p.ld_ids + p.col] = tok;
    p.next[b] = tok;
    p.done[b] = (fin || tok == p.eos) ? 1 : 0;
    if (!fin && tok >= q.ts_begin) q.last_ts[b] = (int)tok;
    if (p.sum_logp && !fin) {
      float lse = ts_l;
      if (!mask_text) {
        float m = a.tm, ss = a.tse;
        if (a.bs > -INFINITY) lse_merge(m, ss, a.bs, a.se);
        lse = lse_val(m, ss);
      }
      p.sum_logp[b] += to_f32(row[best]) - lse;
    }
  }
}

// grid (G, B): G == 1 -> whole row + finish; G > 1 -> partial of slice blockIdx.x into ws
template <typename E>
__global__ __launch_bounds__(256) void greedy_select_ts_kernel(SelTsP q, int slice, float* ws) {
  __shared__ float sv[4][8];
  __shared__ int si[4][2];
  __shared__ float sx[4][4];
  __shared__ int sxi[4][4];
  const int g = blockIdx.x, G = gridDim.x, b = blockIdx.y;
  if (q.s.t_dev) q.s.col += *q.s.t_dev;
  const TsRow r = ts_row(q, b);
  const bool lse = q.s.sum_logp != nullptr;
  const E* row = (const E*)q.s.logits + b * q.s.ld;
  TsAcc a;
  ts_init(a);
  const int lo = G == 1 ? 0 : g * slice, hi = G == 1 ? q.s.V : min(q.s.V, lo + slice);
  ts_scan(q, r, row, a, lo, hi);
  ts_block(a, lse, sv, si);
  if (G == 1) {
    ts_finish<E>(q, r, b, a, sx, sxi);
  } else if (threadIdx.x == 0) {
    float* w = ws + ((int64_t)b * G + g) * SEL_WORDS;
    w[0] = a.bt; w[1] = a.bs; w[2] = a.se; w[3] = a.tm; w[4] = a.tse;
    w[5] = __int_as_float(a.it); w[6] = __int_as_float(a.is);
  }
}

template <typename E>
__global__ __launch_bounds__(256) void ts_merge_kernel(SelTsP q, int G, const float* ws) {
  __shared__ float sx[4][4];
  __shared__ int sxi[4][4];
  const int b = blockIdx.x;
  if (q.s.t_dev) q.s.col += *q.s.t_dev;
  const TsRow r = ts_row(q, b);
  const bool lse = q.s.sum_logp != nullptr;
  TsAcc a;
  ts_init(a);
  if (threadIdx.x == 0)
    for (int g = 0; g < G; ++g) {
      const float* w = ws + ((int64_t)b * G + g) * SEL_WORDS;
      TsAcc o;
      o.bt = w[0]; o.bs = w[1]; o.se = w[2]; o.tm = w[3]; o.tse = w[4];
      o.it = __float_as_int(w[5]); o.is = __float_as_int(w[6]);
      ts_merge(a, o, lse);
    }
  ts_finish<E>(q, r, b, a, sx, sxi);
}

// out[b] = log_softmax(logits[b, :V])[token]   (fp32 of the bf16 / fp32 row)
template <typename E>
__global__ __launch_bounds__(256) void token_logprob_kernel(const E* __restrict__ logits, int64_t ld, int V,
                                                            int token, float* __restrict__ out) {
  __shared__ float sv[4][4];
  const int b = blockIdx.x;
  const E* row = logits + b * ld;
  float m = -INFINITY, s = 0.f;
  for (int v = threadIdx.x; v < V; v += 256) {
    const float x = to_f32(row[v]);
    if (x > -INFINITY) lse_add(m, s, x);
  }
  block_lse(m, s, sv, 0);
  if (threadIdx.x == 0) out[b] = to_f32(row[token]) - lse_val(m, s);
}

// x[b] = tok[ids[b]] + pos[*t_dev]   (decoder input embedding of step t, HF modeling_whisper.py:720-735)
__global__ void embed_step_kernel(const int64_t* __restrict__ ids, const void* __restrict__ tok, int tok_dtype,
                                  const void* __restrict__ pos, int pos_dtype, void* __restrict__ out, int out_dtype,
                                  int D, const int* __restrict__ t_dev) {
  const int b = blockIdx.x;
  const int64_t id = ids[b];
  const int64_t t = *t_dev;
  for (int e = threadIdx.x; e < D; e += blockDim.x) {
    const float s = ld_as_f32(tok, tok_dtype, id * D + e) + ld_as_f32(pos, pos_dtype, t * D + e);
    st_from_f32(out, out_dtype, (int64_t)b * D + e, s);
  }
}

// cache[b][*t_dev][0:n] = src[b][0:n]   (16-B vectors: 8 bf16 or 4 fp32)
template <typename E>
__global__ void kv_append_kernel(const E* __restrict__ src, int64_t ld_src, E* __restrict__ cache,
                                 int64_t ld_row, int64_t sb, int n, const int* __restrict__ t_dev) {
  constexpr int W = 16 / sizeof(E);
  const int b = blockIdx.y;
  const int64_t t = *t_dev;
  const int i = (blockIdx.x * blockDim.x + threadIdx.x) * W;
  if (i < n) *(f32x4*)(cache + b * sb + t * ld_row + i) = *(const f32x4*)(src + b * ld_src + i);
}

__global__ void step_advance_kernel(int* t_dev, int by) {
  if (threadIdx.x == 0) *t_dev += by;
}

// vector row loads when every row starts 16-B aligned and has room for the last 8-id chunk
int sel_vec(const void* logits, int64_t ld, int V) {
  return ((uintptr_t)logits % 16 == 0 && ld % 8 == 0 && ld >= (int64_t)((V + 7) / 8) * 8) ? 1 : 0;
}

// launch K<bf16> or K<float> by the logits dtype code
#define TW_LAUNCH_DT(dt, K, grid, block, ...)                                              \
  do {                                                                                      \
    if ((dt) == TW_BF16) hipLaunchKernelGGL(K<bf16>, grid, block, 0, stream, __VA_ARGS__);   \
    else if ((dt) == TW_F16) hipLaunchKernelGGL(K<f16>, grid, block, 0, stream, __VA_ARGS__);  \
    else if ((dt) == TW_F32) hipLaunchKernelGGL(K<float>, grid, block, 0, stream, __VA_ARGS__); \
    else return TW_EUNSUPPORTED;                                                            \
  } while (0)

// slices per row: enough workgroups to cover the chip for a handful of rows, one per row from 256 rows
// up; the slices are multiples of 8 ids (for_row's 16-B chunks)
int sel_slices(int B, int V) {
  int G = 1;
  while (G < 32 && (int64_t)B * G * 2 <= 512) G *= 2;
  const int slice = ((V + G - 1) / G + 7) / 8 * 8;
  return (V + slice - 1) / slice;
}

int launch_select(const SelP& p, int B, int logits_dtype, hipStream_t stream) {
  const int G = sel_slices(B, p.V);
  const int slice = ((p.V + G - 1) / G + 7) / 8 * 8;
  float* ws = G > 1 ? (float*)tw_device_workspace(stream, (size_t)B * G * SEL_WORDS * sizeof(float)) : nullptr;
  if (G > 1 && ws) {
    TW_LAUNCH_DT(logits_dtype, greedy_select_kernel, dim3(G, B), dim3(256), p, slice, ws);
    TW_LAUNCH_DT(logits_dtype, greedy_merge_kernel, dim3(B), dim3(64), p, G, ws);
  } else {
    TW_LAUNCH_DT(logits_dtype, greedy_select_kernel, dim3(1, B), dim3(256), p, p.V, (float*)nullptr);
  }
  TW_CHECK_LAUNCH();
  return TW_OK;
}

int launch_select_ts(const SelTsP& q, int B, int logits_dtype, hipStream_t stream) {
  const int G = sel_slices(B, q.s.V);
  const int slice = ((q.s.V + G - 1) / G + 7) / 8 * 8;
  float* ws = G > 1 ? (float*)tw_device_workspace(stream, (size_t)B * G * SEL_WORDS * sizeof(float)) : nullptr;
  if (G > 1 && ws) {
    TW_LAUNCH_DT(logits_dtype, greedy_select_ts_kernel, dim3(G, B), dim3(256), q, slice, ws);
    TW_LAUNCH_DT(logits_dtype, ts_merge_kernel, dim3(B), dim3(256), q, G, ws);
  } else {
    TW_LAUNCH_DT(logits_dtype, greedy_select_ts_kernel, dim3(1, B), dim3(256), q, q.s.V, (float*)nullptr);
  }
  TW_CHECK_LAUNCH();
  return TW_OK;
}

}  // namespace

extern "C" int tw_greedy_select_ts(const void* logits, int64_t ld, int logits_dtype, int B, int V, const uint32_t* suppress_bits,
                                   const uint32_t* begin_bits, int64_t eos, uint8_t* done, int64_t* ids, int64_t ld_ids,
                                   int col, int64_t* next_ids, const int* t_dev, int begin_col, int ts_begin,
                                   int no_ts, int max_initial, int* last_ts, hipStream_t stream) {
  if (B <= 0) return TW_OK;
  if (V <= 0 || ld < V || !done || !ids || !next_ids || !last_ts || ts_begin <= eos || ts_begin > V) return TW_EINVAL;
  SelTsP q;
  q.s.logits = logits; q.s.ld = ld; q.s.V = V;
  q.s.suppress = suppress_bits; q.s.begin = begin_bits; q.s.apply_begin = 0;
  q.s.eos = eos; q.s.done = done; q.s.ids = ids; q.s.ld_ids = ld_ids; q.s.col = col; q.s.next = next_ids;
  q.s.t_dev = t_dev; q.s.begin_col = begin_col;
  q.s.ctl = nullptr; q.s.sum_logp = nullptr; q.s.vec = sel_vec(logits, ld, V);
  q.begin_col = begin_col; q.ts_begin = ts_begin; q.no_ts = no_ts; q.max_initial = max_initial; q.last_ts = last_ts;
  return launch_select_ts(q, B, logits_dtype, stream);
}

extern "C" int tw_select_sample_ts(const void* logits, int64_t ld, int logits_dtype, int B, int V, const uint32_t* suppress_bits,
                                   const uint32_t* begin_bits, int64_t eos, uint8_t* done, int64_t* ids, int64_t ld_ids,
                                   int col, int64_t* next_ids, const int* t_dev, int begin_col, int ts_begin,
                                   int no_ts, int max_initial, int* last_ts, const uint32_t* ctl, float* sum_logp,
                                   hipStream_t stream) {
  if (B <= 0) return TW_OK;
  if (V <= 0 || ld < V || !done || !ids || !next_ids || !last_ts || ts_begin <= eos || ts_begin > V) return TW_EINVAL;
  if (B >= (1 << 21) || V >= (1 << 21)) return TW_EUNSUPPORTED;     // RNG key widths
  SelTsP q;
  q.s.logits = logits; q.s.ld = ld; q.s.V = V;
  q.s.suppress = suppress_bits; q.s.begin = begin_bits; q.s.apply_begin = 0;
  q.s.eos = eos; q.s.done = done; q.s.ids = ids; q.s.ld_ids = ld_ids; q.s.col = col; q.s.next = next_ids;
  q.s.t_dev = t_dev; q.s.begin_col = begin_col;
  q.s.ctl = ctl; q.s.sum_logp = sum_logp; q.s.vec = sel_vec(logits, ld, V);
  q.begin_col = begin_col; q.ts_begin = ts_begin; q.no_ts = no_ts; q.max_initial = max_initial; q.last_ts = last_ts;
  return launch_select_ts(q, B, logits_dtype, stream);
}

extern "C" int tw_token_logprob(const void* logits, int64_t ld, int logits_dtype, int B, int V, int token,
                                float* out, hipStream_t stream) {
  if (B <= 0) return TW_OK;
  if (V <= 0 || ld < V || token < 0 || token >= V || !out) return TW_EINVAL;
  if (logits_dtype == TW_BF16)
    hipLaunchKernelGGL(token_logprob_kernel<bf16>, dim3(B), dim3(256), 0, stream, (const bf16*)logits, ld, V, token, out);
  else if (logits_dtype == TW_F16)
    hipLaunchKernelGGL(token_logprob_kernel<f16>, dim3(B), dim3(256), 0, stream, (const f16*)logits, ld, V, token, out);
  else if (logits_dtype == TW_F32)
    hipLaunchKernelGGL(token_logprob_kernel<float>, dim3(B), dim3(256), 0, stream, (const float*)logits, ld, V, token,
                       out);
  else
    return TW_EUNSUPPORTED;
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_embed_step(const int64_t* ids, const void* tok, int tok_dtype, const void* pos, int pos_dtype,
                             void* out, int out_dtype, int B, int D, const int* t_dev, hipStream_t stream) {
  if (B <= 0) return TW_OK;
  if (!t_dev || D <= 0) return TW_EINVAL;
  hipLaunchKernelGGL(embed_step_kernel, dim3(B), dim3(256), 0, stream, ids, tok, tok_dtype, pos, pos_dtype, out,
                     out_dtype, D, t_dev);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

// cross-attention K/V, row-interleaved [rows = B*Tk][ld] (k at columns 0..d, v at d..2d, head h at 64h..) ->
// head-major dst: K [B][H][Tk][64] then V [B][H][Tk][64] (one (clip, head) reads two contiguous Tk*64 runs)
template <typename E>
__global__ void kv_head_major_kernel(const E* __restrict__ src, int64_t ld, E* __restrict__ dst, int Tk, int H,
                                     int64_t rows) {
  constexpr int W = 16 / sizeof(E);
  const int d = H * 64, nv = 2 * d / W;                     // 16-B vectors per source row
  const int64_t total = rows * nv;
  const int64_t half = rows * d;                            // elements of the K part
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / nv;
    const int c = (int)(i - r * nv) * W;                    // source column
    const int part = c >= d, cc = c - part * d, h = cc >> 6, e = cc & 63;
    const int64_t b = r / Tk, t = r - b * Tk;
    const int4 v = *(const int4*)(src + r * ld + c);
    *(int4*)(dst + part * half + ((b * H + h) * Tk + t) * 64 + e) = v;
  }
}

extern "C" int tw_kv_head_major(const void* src, int64_t ld, void* dst, int B, int Tk, int H, int dtype,
                                hipStream_t stream) {
  if (B <= 0 || Tk <= 0 || H <= 0) return TW_OK;
  const int w = dtype == TW_F32 ? 3 : 7;
  if ((ld & w) || ld < 2 * 64 * H || (((uintptr_t)src | (uintptr_t)dst) & 15)) return TW_EINVAL;
  const int64_t rows = (int64_t)B * Tk;
  const int64_t nvec = rows * (2 * 64 * H) / (w + 1);
  const dim3 grid((unsigned)std::min<int64_t>((nvec + 255) / 256, 16384));
  if (dtype == TW_BF16 || dtype == TW_F16)
    hipLaunchKernelGGL(kv_head_major_kernel<bf16>, grid, dim3(256), 0, stream, (const bf16*)src, ld, (bf16*)dst, Tk, H,
                       rows);
  else if (dtype == TW_F32)
    hipLaunchKernelGGL(kv_head_major_kernel<float>, grid, dim3(256), 0, stream, (const float*)src, ld, (float*)dst,
                       Tk, H, rows);
  else
    return TW_EUNSUPPORTED;
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_kv_append(const void* src, int64_t ld_src, void* cache, int64_t ld_row, int64_t sb, int B, int n,
                            int dtype, const int* t_dev, hipStream_t stream) {
  if (B <= 0 || n <= 0) return TW_OK;
  const int w = dtype == TW_F32 ? 3 : 7;          // 16-B vectors: 4 fp32 / 8 bf16
  if (!t_dev || (n & w) || (ld_src & w) || (ld_row & w) || (sb & w) || (((uintptr_t)src | (uintptr_t)cache) & 15))
    return TW_EINVAL;
  if (dtype == TW_BF16 || dtype == TW_F16)
    hipLaunchKernelGGL(kv_append_kernel<bf16>, dim3((n / 8 + 255) / 256, B), dim3(256), 0, stream, (const bf16*)src,
                       ld_src, (bf16*)cache, ld_row, sb, n, t_dev);
  else if (dtype == TW_F32)
    hipLaunchKernelGGL(kv_append_kernel<float>, dim3((n / 4 + 255) / 256, B), dim3(256), 0, stream, (const float*)src,
                       ld_src, (float*)cache, ld_row, sb, n, t_dev);
  else
    return TW_EUNSUPPORTED;
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_step_advance(int* t_dev, int by, hipStream_t stream) {
  if (!t_dev) return TW_EINVAL;
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(64), 0, stream, t_dev, by);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_decode_attn_hs(const void* q, int64_t sqb, const void* k, int64_t ldk, int64_t skb, int64_t hsk,
                                 const void* v, int64_t ldv, int64_t svb, int64_t hsv, void* o, int64_t sob, int B,
                                 int H, int Tk, const int* tk_dev, int head_dim, float scale, int dtype,
                                 hipStream_t stream) {
  if (head_dim != 64) return TW_EUNSUPPORTED;
  if (B <= 0 || H <= 0) return TW_OK;
  if ((!tk_dev && Tk <= 0) || Tk > DA_MAX_TK) return TW_EUNSUPPORTED;
  if (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v) & 15) return TW_EINVAL;
  if ((sqb | ldk | skb | ldv | svb | hsk | hsv) & 7) return TW_EINVAL;
  if (skb < 0 || svb < 0 || hsk < 0 || hsv < 0) return TW_EINVAL;
  DecP p;
  if (dtype == TW_F32 && ((sqb | ldk | skb | ldv | svb) & 3)) return TW_EINVAL;
  p.q = q; p.sqb = sqb;
  p.k = k; p.ldk = ldk; p.skb = skb;
  p.v = v; p.ldv = ldv; p.svb = svb;
  p.o = o; p.sob = sob;
  p.hsk = hsk; p.hsv = hsv;
  p.H = H; p.Tk = Tk; p.tk_dev = tk_dev; p.c = scale * 1.4426950408889634f;
  // few (clip, head) pairs (batch-1 long-form, small batches): split the keys into chunks of DA_SPLIT over
  // the grid's y dimension, then combine.  Measured (tools/bench_decode_attn.py, H = 20, Tk = 1500): B = 1
  // 26.9 -> 14.6 us, B = 16 46.9 -> 31.2 us; from B = 64 (1280 pairs) the one-workgroup-per-pair kernel is
  // faster (90.6 vs 114.8 us).  With tk_dev (self-attention over a graph-captured cache) the host does
  // not know Tk, so the chunks would have to cover the kernel's DA_MAX_TK bound: measured on c5 (batch-1
  // long-form, Tk <= 448) that costs more than it saves (2.75 -> 2.93 ms per decode step), so only fixed-Tk calls
  // below 640 pairs split.
  const int nchunk = (Tk + DA_SPLIT - 1) / DA_SPLIT;
  const bool split = !tk_dev && B * H < 640;
  if (split && nchunk >= 2 && nchunk <= DA_MAX_CHUNK) {
    float* ws = (float*)tw_device_workspace(stream, (size_t)B * H * nchunk * 66 * sizeof(float));
    if (ws) {
      TW_LAUNCH_DT(dtype, decode_attn_split_kernel, dim3(B * H, nchunk), dim3(DA_THREADS), p, DA_SPLIT, ws);
      TW_LAUNCH_DT(dtype, decode_attn_combine_kernel, dim3(B * H), dim3(64), p, nchunk, ws);
      TW_CHECK_LAUNCH();
      return TW_OK;
    }
  }
  if (B * H >= DA_BIG) TW_LAUNCH_DT(dtype, decode_attn_u2_kernel, dim3(B * H), dim3(DA_THREADS), p);
  else TW_LAUNCH_DT(dtype, decode_attn_u4_kernel, dim3(B * H), dim3(DA_THREADS), p);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_decode_attn(const void* q, int64_t sqb, const void* k, int64_t ldk, int64_t skb, const void* v,
                              int64_t ldv, int64_t svb, void* o, int64_t sob, int B, int H, int Tk, const int* tk_dev,
                              int head_dim, float scale, int dtype, hipStream_t stream) {
  return tw_decode_attn_hs(q, sqb, k, ldk, skb, 64, v, ldv, svb, 64, o, sob, B, H, Tk, tk_dev, head_dim, scale, dtype,
                           stream);
}

extern "C" int tw_greedy_select(const void* logits, int64_t ld, int logits_dtype, int B, int V, const uint32_t* suppress_bits,
                                const uint32_t* begin_bits, int apply_begin, int64_t eos, uint8_t* done, int64_t* ids,
                                int64_t ld_ids, int col, int64_t* next_ids, const int* t_dev, int begin_col,
                                hipStream_t stream) {
  if (B <= 0) return TW_OK;
  if (V <= 0 || ld < V || !done || !ids || !next_ids) return TW_EINVAL;
  SelP p;
  p.logits = logits; p.ld = ld; p.V = V;
  p.suppress = suppress_bits; p.begin = begin_bits; p.apply_begin = apply_begin;
  p.eos = eos; p.done = done; p.ids = ids; p.ld_ids = ld_ids; p.col = col; p.next = next_ids;
  p.t_dev = t_dev; p.begin_col = begin_col;
  p.ctl = nullptr; p.sum_logp = nullptr; p.vec = sel_vec(logits, ld, V);
  return launch_select(p, B, logits_dtype, stream);
}

extern "C" int tw_select_sample(const void* logits, int64_t ld, int logits_dtype, int B, int V, const uint32_t* suppress_bits,
                                const uint32_t* begin_bits, int apply_begin, int64_t eos, uint8_t* done, int64_t* ids,
                                int64_t ld_ids, int col, int64_t* next_ids, const int* t_dev, int begin_col,
                                const uint32_t* ctl, float* sum_logp, hipStream_t stream) {
  if (B <= 0) return TW_OK;
  if (V <= 0 || ld < V || !done || !ids || !next_ids) return TW_EINVAL;
  if (B >= (1 << 21) || V >= (1 << 21)) return TW_EUNSUPPORTED;     // RNG key widths
  SelP p;
  p.logits = logits; p.ld = ld; p.V = V;
  p.suppress = suppress_bits; p.begin = begin_bits; p.apply_begin = apply_begin;
  p.eos = eos; p.done = done; p.ids = ids; p.ld_ids = ld_ids; p.col = col; p.next = next_ids;
  p.t_dev = t_dev; p.begin_col = begin_col;
  p.ctl = ctl; p.sum_logp = sum_logp; p.vec = sel_vec(logits, ld, V);
  return launch_select(p, B, logits_dtype, stream);
}
