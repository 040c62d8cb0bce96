// nais_pairs.hip -- the "pairs" strategy of full-catalog scoring.
//
// Every term of a user's score, for history item j and candidate c (validation.py:11-27 over
// model.py:57-89), depends on (j, c) only:
//   e_jc = exp(w2 . ReLU(W1 (h_j (.) t_c) + b1)) [j != c],   s_jc = h_j . t_c
//   logit_uc = sum_{j in H_u} e_jc s_jc / (sum_{j in H_u} e_jc)^beta
// At the bench geometry each (j, c) pair is shared by sum_u h_u / P ~ 50 users, so the catalog
// kernels in pair-table mode (nais_pair_table) evaluate the MLP once per pair of the users'
// distinct history items x a column block of candidates, and this file's pair_gather_kernel
// forms each user's N = sum e s and S = sum e by streaming the user's h_u table rows from HBM
// (coalesced 16-byte loads; the history-gather kernel of the north star). Same per-pair
// arithmetic, same j order of the sums as the direct kernels.
//
//   nais_pair_rows    distinct history items of a user list -> items[] + rowmap[P] (POI -> row)
//   nais_pair_gather  per user: scores[c] for c in a column block from the tables
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <string>

#include "nais.h"
#include "nais_internal.h"
#include "nais_geo.h"

namespace {

// Columns per lane: stripe = 64 * CPL columns. (A/B, profiles/r1/: 2 columns per lane -- a
// 128-column stripe -- 654 vs 560 ms per job, 8 per lane -- 512 columns, 410 MB of stripe, past
// the Infinity Cache -- 845 ms; non-temporal table loads -15 %, non-temporal score stores +-1 %.)
constexpr int CPL = 4;
typedef float nfv __attribute__((ext_vector_type(CPL)));
typedef double ndv __attribute__((ext_vector_type(CPL)));

__device__ __forceinline__ nfv loadv(const float* p) { return *reinterpret_cast<const nfv*>(p); }

constexpr int SCAN_THREADS = 1024;

__global__ void mark_kernel(const int64_t* __restrict__ indptr, const int64_t* __restrict__ indices,
                            const int32_t* __restrict__ users, int32_t* __restrict__ flag) {
  const int64_t u = users[blockIdx.x];
  for (int64_t i = indptr[u] + threadIdx.x; i < indptr[u + 1]; i += blockDim.x) flag[indices[i]] = 1;
}

__device__ __forceinline__ int block_excl_scan(int v, int* sh, int& total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int q = 0; q < SCAN_THREADS / 64; ++q) {
      const int t = sh[q];
      sh[q] = run;
      run += t;
    }
    sh[SCAN_THREADS / 64] = run;
  }
  __syncthreads();
  total = sh[SCAN_THREADS / 64];
  const int r = x - v + sh[w];
  __syncthreads();
  return r;
}

// per-block counts of flagged POIs
__global__ void __launch_bounds__(SCAN_THREADS)
count_kernel(const int32_t* __restrict__ flag, int64_t P, int32_t* __restrict__ bsum) {
  __shared__ int sh[SCAN_THREADS / 64 + 1];
  const int64_t p = int64_t(blockIdx.x) * SCAN_THREADS + threadIdx.x;
  int total;
  block_excl_scan(p < P ? flag[p] : 0, sh, total);
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// exclusive scan of the block counts (one workgroup, any number of blocks)
__global__ void __launch_bounds__(SCAN_THREADS)
scan_blocks_kernel(int32_t* __restrict__ bsum, int64_t nb, int64_t* __restrict__ count) {
  __shared__ int sh[SCAN_THREADS / 64 + 1];
  int64_t run = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += SCAN_THREADS) {
    const int64_t b = b0 + threadIdx.x;
    const int v = b < nb ? bsum[b] : 0;
    int total;
    const int ex = block_excl_scan(v, sh, total);
    if (b < nb) bsum[b] = int32_t(run + ex);
    run += total;
  }
  if (threadIdx.x == 0) *count = run;
}

// rowmap[p] = row of POI p in items[] (ascending POI order), -1 if p is in no history
__global__ void __launch_bounds__(SCAN_THREADS)
place_kernel(int32_t* __restrict__ flag_rowmap, int64_t P, const int32_t* __restrict__ bsum,
             int64_t* __restrict__ items) {
  __shared__ int sh[SCAN_THREADS / 64 + 1];
  const int64_t p = int64_t(blockIdx.x) * SCAN_THREADS + threadIdx.x;
  const int f = p < P ? flag_rowmap[p] : 0;
  int total;
  const int ex = block_excl_scan(f, sh, total);
  if (p < P) {
    const int row = bsum[blockIdx.x] + ex;
    flag_rowmap[p] = f ? row : -1;
    if (f) items[row] = p;
  }
}

// One wave per user, 4 users per workgroup; a wave covers a 256-column stripe (CPL = 4 columns
// per lane). Grid x = user groups (fastest), y = stripes: the workgroups in flight read the same
// stripe of the tables -- J x 256 x 8 B, ~200 MB at J = 100k -- so the Infinity Cache serves the
// rows the ~50 users sharing each item read (A/B: profiles/r1/pairs/). N and S are summed in
// history (CSR) order, then the score of model.py:55 / validation.py:26; history POIs get -1.
constexpr int GW = 4;                       // users (waves) per workgroup (1 / 2 / 8: +-1 %)

// lane jj's 64-bit value, as a wave-uniform scalar (readlane returns int: widen via uint32_t)
__device__ __forceinline__ int64_t bcast64(uint32_t lo, uint32_t hi, int jj) {
  const uint32_t l = uint32_t(__builtin_amdgcn_readlane(int(lo), jj));
  const uint32_t h = uint32_t(__builtin_amdgcn_readlane(int(hi), jj));
  return int64_t((uint64_t(h) << 32) | uint64_t(l));
}
constexpr int STRIPE = 64 * CPL;             // columns per wave

// Rows issued ahead per wave in the gather loops. A plain `#pragma unroll` over a runtime trip
// count does not unroll here (the loop holds convergent readlanes), which left one row -- 2 KB per
// wave -- in flight and the gather latency-bound; GU explicit loads per step keep GU rows in flight
// while the adds stay in history (CSR) order.
constexpr int GU = 8;   // config-4 job at 4 / 8 / 12 / 16 rows: 0.607 / 0.597 / 0.606 / 0.657 s (profiles/r5/gu)

// CPL columns of one table row for a lane with nv valid columns (CPL: one vector load; fewer, the
// last lane of a block whose width is not a multiple of CPL: scalar loads, 0 past the block).
template <typename V, typename T>
__device__ __forceinline__ V load_cols(const T* __restrict__ p, int nv) {
  if (nv == CPL) return *reinterpret_cast<const V*>(p);
  V v;
#pragma unroll
  for (int q = 0; q < CPL; ++q) v[q] = q < nv ? p[q] : T(0);
  return v;
}

// Sa += Σ E[row(j), x..x+CPL), Na += Σ ES[...] over the jn (wave-uniform) rows whose offsets the
// lanes 0..jn-1 hold in (mlo, mhi), in lane order; nv = this lane's valid columns (0..CPL; past
// them the sums get +0). Every readlane runs with the whole wave active: a readlane inside a
// branch on nv could read a lane's register after that lane's side of the branch reused it (the
// register allocator only keeps values live for the lanes a branch runs), which gave the last
// lane of an odd-width block wrong rows.
__device__ __forceinline__ void gather_rows(const float* __restrict__ E, const float* __restrict__ ES,
                                            uint32_t mlo, uint32_t mhi, int jn, int64_t x, int nv,
                                            float (&Sa)[CPL], float (&Na)[CPL]) {
  int jj = 0;
  for (; jj + GU <= jn; jj += GU) {
    int64_t o[GU];
#pragma unroll
    for (int g = 0; g < GU; ++g) o[g] = bcast64(mlo, mhi, jj + g) + x;
    nfv e[GU], t[GU];
#pragma unroll
    for (int g = 0; g < GU; ++g) {
      e[g] = load_cols<nfv>(E + o[g], nv);
      t[g] = load_cols<nfv>(ES + o[g], nv);
    }
#pragma unroll
    for (int g = 0; g < GU; ++g)
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        Sa[q] += e[g][q];
        Na[q] += t[g][q];
      }
  }
  for (; jj < jn; ++jj) {
    const int64_t o = bcast64(mlo, mhi, jj) + x;
    const nfv e = load_cols<nfv>(E + o, nv);
    const nfv t = load_cols<nfv>(ES + o, nv);
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      Sa[q] += e[q];
      Na[q] += t[q];
    }
  }
}

__device__ __forceinline__ int valid_cols(int64_t x, int64_t cols) {
  return x >= cols ? 0 : (x + CPL <= cols ? CPL : int(cols - x));
}

__global__ void __launch_bounds__(GW * 64)
pair_gather_kernel(const float* __restrict__ E, const float* __restrict__ ES, int64_t ld,
                   const int32_t* __restrict__ rowmap, const int64_t* __restrict__ indptr,
                   const int64_t* __restrict__ indices, const int32_t* __restrict__ users,
                   int32_t nusers, int64_t col0, int64_t cols, float beta,
                   float* __restrict__ scores, int64_t score_ld, int64_t score_col0,
                   int32_t* __restrict__ nan_count) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: scalar user loads
  const int64_t slot = int64_t(blockIdx.x) * GW + w;
  if (slot >= nusers) return;                // wave-uniform; no workgroup barriers below
  const int64_t u = users[slot];
  const int64_t hb = indptr[u], hl = indptr[u + 1] - hb;
  const int64_t x = int64_t(blockIdx.y) * STRIPE + lane * CPL;   // column within the block
  const int nv = valid_cols(x, cols);
  float Sa[CPL], Na[CPL];
#pragma unroll
  for (int q = 0; q < CPL; ++q) Sa[q] = Na[q] = 0.f;
  for (int64_t j0 = 0; j0 < hl; j0 += 64) {
    const int jn = __builtin_amdgcn_readfirstlane((int)std::min<int64_t>(64, hl - j0));
    // row offsets of 64 history items, one per lane, broadcast with readlane below
    const int64_t mine = lane < jn ? int64_t(rowmap[indices[hb + j0 + lane]]) * ld : 0;
    const uint32_t mlo = uint32_t(mine), mhi = uint32_t(mine >> 32);
    gather_rows(E, ES, mlo, mhi, jn, x, nv, Sa, Na);
  }
  float* out = scores + slot * score_ld + (col0 - score_col0) + x;
  int nan = 0;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    if (x + q < cols) {
      float logit = 0.f;   // empty history: logit 0
      if (hl > 0) logit = Na[q] / ((beta == 0.5f) ? sqrtf(Sa[q]) : powf(Sa[q], beta));
      float sc = 1.0f / (1.0f + expf(-logit));
      if (logit != logit) {
        sc = __builtin_nanf("");
        ++nan;
      }
      out[q] = sc;
    }
  }
  __threadfence_block();   // this wave's score stores land before its -1 stores below
  const int64_t lo = col0 + int64_t(blockIdx.y) * STRIPE;
  const int64_t hi = std::min<int64_t>(lo + STRIPE, col0 + cols);
  for (int64_t j = lane; j < hl; j += 64) {
    const int64_t c = indices[hb + j];
    if (c >= lo && c < hi) {
      float* o = scores + slot * score_ld + (c - score_col0);
      if (*o != *o) --nan;   // counted above, but not a candidate
      *o = -1.f;
    }
  }
  if (nan_count) {
    for (int o = 32; o > 0; o >>= 1) nan += __shfl_xor(nan, o);
    if (lane == 0 && nan) atomicAdd(nan_count, nan);
  }
}

// ---------------------------------------------------------------------------------------------
// Fused gather + running top-k (validation.py:26-27 without the [users, P] score rows).
// Same sums and score arithmetic as pair_gather_kernel, one launch per 256-column stripe (so the
// user's list below has one writer per launch). Each user keeps its best k keys so far,
//   key = ordered(score) << 32 | (0xFFFFFFFF - poi)     (unique: (score desc, id asc), NaN first)
// sorted descending in keys[slot * k ...] with kcount[slot] of them valid. A wave offers its
// stripe's candidates (history POIs excluded) that beat the current k-th key; if any do, it merges
// them with the list in LDS (bitonic, <= k + 256 keys) and writes the new list back. After the
// first few stripes almost no candidate beats the k-th key, so most waves write nothing.
constexpr int TK_LDS = 512;                 // keys per wave in LDS: k + 256 <= 512  (k <= 256)

__device__ __forceinline__ uint32_t ord_f32_p(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_f32_p(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ void __launch_bounds__(GW * 64)
pair_gather_topk_kernel(const float* __restrict__ E, const float* __restrict__ ES, int64_t ld,
                        const int32_t* __restrict__ rowmap, const int64_t* __restrict__ indptr,
                        const int64_t* __restrict__ indices, const int32_t* __restrict__ users,
                        int32_t nusers, int64_t col0, int64_t cols, float beta, int k,
                        unsigned long long* __restrict__ keys, int32_t* __restrict__ kcount,
                        int32_t* __restrict__ nan_count, int32_t* __restrict__ work) {
  __shared__ unsigned long long lk[GW][TK_LDS];
  __shared__ uint32_t hm[GW][STRIPE / 32];   // history POIs of this stripe, one bit per column
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // work != null: a work queue -- every wave takes user slots from the counter until they run out,
  // so a shader engine with fewer enabled CUs takes fewer (no 32-CU steps in the stream split)
  constexpr int GQ = 4;   // slots per grab: a quarter of the atomics on the one counter
  int64_t qnext = 0, qend = 0;
  for (int64_t it = 0;; ++it) {
  int64_t slot;
  if (work) {
    if (qnext == qend) {
      int got = 0;
      if (lane == 0) got = atomicAdd(work, GQ);
      qnext = __builtin_amdgcn_readfirstlane(got);
      qend = qnext + GQ;
    }
    slot = qnext++;
  } else {
    if (it > 0) break;
    slot = int64_t(blockIdx.x) * GW + w;
  }
  if (slot >= nusers) break;                 // wave-uniform; no workgroup barriers below
  const int64_t u = users[slot];
  const int64_t hb = indptr[u], hl = indptr[u + 1] - hb;
  const int64_t x = int64_t(lane) * CPL;     // column within the stripe [col0, col0 + cols)
  const int nv = valid_cols(x, cols);
  if (lane < STRIPE / 32) hm[w][lane] = 0u;
  wave_lds_sync();
  float Sa[CPL], Na[CPL];
#pragma unroll
  for (int q = 0; q < CPL; ++q) Sa[q] = Na[q] = 0.f;
  for (int64_t j0 = 0; j0 < hl; j0 += 64) {
    const int jn = __builtin_amdgcn_readfirstlane((int)std::min<int64_t>(64, hl - j0));
    int64_t mine = 0;
    if (lane < jn) {
      const int64_t c = indices[hb + j0 + lane];
      mine = int64_t(rowmap[c]) * ld;
      const int64_t r = c - col0;
      if (r >= 0 && r < cols) atomicOr(&hm[w][r >> 5], 1u << (r & 31));
    }
    const uint32_t mlo = uint32_t(mine), mhi = uint32_t(mine >> 32);
    gather_rows(E, ES, mlo, mhi, jn, x, nv, Sa, Na);
  }
  wave_lds_sync();
  // the wave's candidates and the current k-th key
  const int cnt = kcount[slot];
  const unsigned long long thr = cnt == k ? keys[slot * k + k - 1] : 0ull;   // valid keys are > 0
  unsigned long long kq[CPL];
  uint32_t offer = 0;   // bit q: column x + q is offered
  int nan = 0;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    kq[q] = 0ull;
    const int64_t r = x + q;
    if (r < cols && !((hm[w][r >> 5] >> (r & 31)) & 1u)) {
      float logit = 0.f;   // empty history: logit 0
      if (hl > 0) logit = Na[q] / ((beta == 0.5f) ? sqrtf(Sa[q]) : powf(Sa[q], beta));
      float sc = 1.0f / (1.0f + expf(-logit));
      if (logit != logit) {
        sc = __builtin_nanf("");
        ++nan;
      }
      kq[q] = ((unsigned long long)ord_f32_p(sc) << 32) |
              (unsigned long long)(0xFFFFFFFFu - (uint32_t)(col0 + r));
      if (kq[q] > thr) offer |= 1u << q;
    }
  }
  if (nan_count) {
    for (int o = 32; o > 0; o >>= 1) nan += __shfl_xor(nan, o);
    if (lane == 0 && nan) atomicAdd(nan_count, nan);
  }
  const int mine_n = __popc(offer);
  int excl = mine_n;   // inclusive scan over lanes, then exclusive
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(excl, o);
    if (lane >= o) excl += y;
  }
  const int m = __shfl(excl, 63);
  excl -= mine_n;
  if (m == 0) continue;
  unsigned long long* L = lk[w];
  for (int i = lane; i < cnt; i += 64) L[i] = keys[slot * k + i];
  int pos = cnt + excl;
#pragma unroll
  for (int q = 0; q < CPL; ++q)
    if ((offer >> q) & 1u) L[pos++] = kq[q];
  const int n = cnt + m;
  int n2 = 64;
  while (n2 < n) n2 <<= 1;
  for (int i = n + lane; i < n2; i += 64) L[i] = 0ull;
  wave_lds_sync();
  // bitonic sort, descending
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = lane; i < n2; i += 64) {
        const int partner = i ^ stride;
        if (partner > i) {
          const bool desc = (i & size) == 0;
          const unsigned long long a = L[i], b = L[partner];
          if (desc ? (a < b) : (a > b)) {
            L[i] = b;
            L[partner] = a;
          }
        }
      }
      wave_lds_sync();
    }
  }
  const int nk = n < k ? n : k;
  for (int i = lane; i < nk; i += 64) keys[slot * k + i] = L[i];
  if (lane == 0) kcount[slot] = nk;
  wave_lds_sync();   // the next slot's hm / lk writers after this slot's readers
  }
}


// ---------------------------------------------------------------------------------------------
// Power-law prior on the pairs route (powerLaw.py:86-92, run.py:537-539): pr_d(dist(j, c)) depends
// on the pair only, so it is tabled once per (distinct history POI, candidate) like e and e*s,
// and each user's G[c] = prod_j pr_d(dist(j, c)) is gathered as a float64 product in CSR order --
// the operation order of prior_kernel (nais_powerlaw_prior), hence the same bits.
constexpr int PRIOR_TAB_THREADS = 256;

// pr[r * ld + c - col0] = pr_d(dist(items[r], c)) for r < nitems, c in [col0, col0 + cols)
__global__ void __launch_bounds__(PRIOR_TAB_THREADS)
prior_pair_table_kernel(const double* __restrict__ coords, const int64_t* __restrict__ items,
                        int64_t nitems, int64_t col0, int64_t cols, double a, double b,
                        double* __restrict__ pr, int64_t ld) {
  constexpr int RB = 16;                     // item rows per workgroup (Geo of each in LDS)
  __shared__ Geo hg[RB];
  const int64_t x = int64_t(blockIdx.x) * PRIOR_TAB_THREADS + threadIdx.x;
  const int64_t r0 = int64_t(blockIdx.y) * RB;
  const int rn = (int)std::min<int64_t>(RB, nitems - r0);
  if (threadIdx.x < rn) {
    const int64_t it = items[r0 + threadIdx.x];
    hg[threadIdx.x] = make_geo(coords[2 * it], coords[2 * it + 1]);
  }
  __syncthreads();
  if (x >= cols) return;
  const int64_t c = col0 + x;
  const Geo gc = make_geo(coords[2 * c], coords[2 * c + 1]);
  for (int r = 0; r < rn; ++r) pr[(r0 + r) * ld + x] = ref_pr_d(a, b, ref_dist(hg[r], gc));
}

// G[slot * g_ld + c - g_col0] = prod_j pr[row(j), c] over the user's history in CSR order (1.0 for
// an empty history, -1.0 for history POIs), and gmax[slot] = max(gmax[slot], max over the block's
// candidates) as u64 bits (non-negative doubles order as their bits). One wave per user, 4
// columns per lane, 4 users per workgroup -- the layout of pair_gather_topk_kernel.
// zero_exit: every pr entry is finite (the caller's (a, b) guarantee it), so a product that has
// underflowed to 0.0 stays 0.0 (powerLaw.py:92's np.prod does the same): once all of a wave's
// columns are 0 its remaining rows are not read (long histories underflow: each factor is ~1e-3
// at city distances, so G reaches 0 after ~110 history POIs). The history bitmap is still built.
__global__ void __launch_bounds__(GW * 64)
prior_pair_gather_kernel(const double* __restrict__ pr, int64_t ld, const int32_t* __restrict__ rowmap,
                         const int64_t* __restrict__ indptr, const int64_t* __restrict__ indices,
                         const int32_t* __restrict__ users, int32_t nusers, int64_t col0, int64_t cols,
                         double* __restrict__ G, int64_t g_ld, int64_t g_col0,
                         unsigned long long* __restrict__ gmax, int zero_exit) {
  __shared__ uint32_t hm[GW][STRIPE / 32];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t slot = int64_t(blockIdx.x) * GW + w;
  if (slot >= nusers) return;                // wave-uniform; no workgroup barriers below
  const int64_t u = users[slot];
  const int64_t hb = indptr[u], hl = indptr[u + 1] - hb;
  const int64_t s0 = int64_t(blockIdx.y) * STRIPE;          // this wave's stripe in the block
  const int64_t x = s0 + int64_t(lane) * CPL;
  const int nv = valid_cols(x, cols);
  if (lane < STRIPE / 32) hm[w][lane] = 0u;
  wave_lds_sync();
  double g[CPL];
#pragma unroll
  for (int q = 0; q < CPL; ++q) g[q] = (x + q < cols) ? 1.0 : 0.0;   // columns past the block: 0
  bool all_zero = false;   // wave-uniform: every column's product is 0.0 (zero_exit only)
  for (int64_t j0 = 0; j0 < hl; j0 += 64) {
    const int jn = __builtin_amdgcn_readfirstlane((int)std::min<int64_t>(64, hl - j0));
    int64_t mine = 0;
    if (lane < jn) {
      const int64_t c = indices[hb + j0 + lane];
      mine = int64_t(rowmap[c]) * ld;
      const int64_t r = c - col0 - s0;
      if (r >= 0 && r < STRIPE && r + s0 < cols) atomicOr(&hm[w][r >> 5], 1u << (r & 31));
    }
    if (all_zero) continue;   // only the bitmap is left to build (wave-uniform)
    const uint32_t mlo = uint32_t(mine), mhi = uint32_t(mine >> 32);
    int jj = 0;
    // GU rows' loads in flight (as gather_rows), products still in CSR order; readlanes and the
    // ballot with the whole wave active (columns past the block hold 0.0 and stay 0.0)
    for (; jj + GU <= jn; jj += GU) {
      int64_t o[GU];
#pragma unroll
      for (int u2 = 0; u2 < GU; ++u2) o[u2] = bcast64(mlo, mhi, jj + u2) + x;
      ndv rv[GU];
#pragma unroll
      for (int u2 = 0; u2 < GU; ++u2) rv[u2] = load_cols<ndv>(pr + o[u2], nv);
#pragma unroll
      for (int u2 = 0; u2 < GU; ++u2)
#pragma unroll
        for (int q = 0; q < CPL; ++q) g[q] = __dmul_rn(g[q], rv[u2][q]);
      if (zero_exit) {
        bool nz = false;
#pragma unroll
        for (int q = 0; q < CPL; ++q) nz |= g[q] != 0.0;
        if (__ballot(nz) == 0ull) {
          all_zero = true;
          break;
        }
      }
    }
    if (all_zero) continue;
    for (; jj < jn; ++jj) {
      const ndv rv = load_cols<ndv>(pr + bcast64(mlo, mhi, jj) + x, nv);
#pragma unroll
      for (int q = 0; q < CPL; ++q) g[q] = __dmul_rn(g[q], rv[q]);
    }
    if (zero_exit) {
      bool nz = false;
#pragma unroll
      for (int q = 0; q < CPL; ++q) nz |= g[q] != 0.0;
      all_zero = __ballot(nz) == 0ull;
    }
  }
  wave_lds_sync();
  double m = -1.0;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int64_t xr = x + q;
    if (xr < cols) {
      const int64_t r = xr - s0;
      const bool hist = (hm[w][r >> 5] >> (r & 31)) & 1u;
      const double v = hist ? -1.0 : g[q];
      G[slot * g_ld + (col0 - g_col0) + xr] = v;
      m = fmax(m, v);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
  if (lane == 0 && m >= 0.0) atomicMax(gmax + slot, (unsigned long long)__double_as_longlong(m));
}

// ---------------------------------------------------------------------------------------------
// Bounded gather + exact refine: the fused top-k of pair_gather_topk_kernel from half its bytes.
// The tables are split16 (nais_pair_table_split, nais_internal.h): hi[r, c] = the top 16 bits of
// e and of e*s, ex[r, c] = the exact (e, e*s) pair. Phase 1 (pair_bound_topk_kernel, one launch per
// column block) streams only the hi rows -- 4 bytes per (user, history item, candidate) instead
// of 8 -- and sums, per candidate, S^ = sum e^, N^ = sum es~ and A^ = sum |es~| of the truncated
// values (e^ <= e < e^ (1 + 2^-7); |e*s - es~| < 2^-7 |es~|, see bound_rows), which bound the
// exact fp32 sums the exact gather forms:
//   Sa in [S^ (1 - 3g), S^ (1 + 2^-7)(1 + 3g)],  |Na - N^| <= (2^-7 + 4g) A^,
// g = h 2^-23 + 2^-20 (the fp32 rounding of either h-term sequential sum, twice over), hence an
// interval [lo, hi] around the exact score sigmoid(Na / Sa^beta) (widened by 2^-19 in the logit
// and 2^-20 in the score for the fp32 evaluation of both; a lower logit bound >= 17 means the
// exact score is 1.0f). Each user keeps the top k LOWER bounds so far (lo_keys: its k-th is a
// threshold tau that only grows) and appends every candidate whose UPPER bound reaches tau to a
// survivor list (compacted by the current tau when full; a user whose list overflows is marked
// -1 and refined over the whole column range). A candidate of the exact top k has exact key >=
// the k-th exact key >= the final tau (k candidates have exact key >= their lower bound >= tau),
// so its upper bound reaches every tau on the way: it is a survivor. Phase 2
// (pair_refine_topk_kernel) recomputes, for each survivor with upper key >= the final tau, the
// exact Na and Sa in history (CSR) order -- the exact gather's operations on the
// same fp32 bits, read as one (e, e*s) pair per row from the ex table -- and ranks them: the same
// top-k lists, ids and score bits, as the exact gather.
// Keys as pair_gather_topk_kernel: ordered(score) << 32 | (0xFFFFFFFF - poi).
// Rows in flight per bounded-gather wave. 4: 116 VGPRs, 4 waves per SIMD; 8 held 148 VGPRs, 3 waves.
// Its chain of dependent loads per user (span, ids and rows, list state) hides better with more
// waves. Per launch 2.224 -> 2.168 ms at config 4 and 2.45 -> 2.28 ms on one rank of N = 8, in
// interleaved runs (profiles/r6/chains_ab). Performance only: A/B builds may set it.
#ifndef NAIS_PAIRS_BGU
#define NAIS_PAIRS_BGU 4
#endif
constexpr int BGU = NAIS_PAIRS_BGU;
constexpr int BCPL = 8;                       // columns per lane: 32-byte hi rows per lane
constexpr int BSTRIPE = 64 * BCPL;            // 512 columns per wave (one launch per block)
constexpr int BK_LDS = 512;                   // keys per wave in LDS: k + 256 offered (k <= 256)

typedef float f2v __attribute__((ext_vector_type(2)));

// S^ += e^, N^ += es~, A^ += |es~| over the jn rows whose item rows lanes 0..jn-1 hold (CSR order).
// e^ = hi << 16 is e truncated to its top 16 bits; es~ is the hi word itself read as a float: the
// top 16 bits of e*s followed by those of e, so |es~| and |e*s| both lie in [|es^|, |es^| + ulp16)
// with the sign of e*s -- |e*s - es~| < 2^-7 |es~|, the bound the refine threshold assumes. Rows
// are read through a buffer resource on the row's base (scalar: readlane of the row, s_mul) with
// the lane's constant column offset, so a row costs no VALU for its address, and the bytes past
// the launch's columns read as 0 (num_records), which adds nothing. S and N take v_pk_add_f32.
__device__ __forceinline__ void bound_rows(const uint32_t* __restrict__ HI, int64_t ld, int32_t mrow,
                                           int jn, uint32_t colbytes, uint32_t voff, f2v (&S)[BCPL / 2],
                                           f2v (&N)[BCPL / 2], float (&A)[BCPL]) {
  auto row = [&](int jj) __attribute__((always_inline)) {
    const int64_t r = __builtin_amdgcn_readlane(mrow, jj);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(HI) + r * ld, (short)0, (int)colbytes,
                                             0x00020000);
  };
  auto acc = [&](const uint4 (&v)[2]) __attribute__((always_inline)) {
    const uint32_t w[BCPL] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
#pragma unroll
    for (int q = 0; q < BCPL; q += 2) {
      S[q / 2] += f2v{__uint_as_float(w[q] << 16), __uint_as_float(w[q + 1] << 16)};
      N[q / 2] += f2v{__uint_as_float(w[q]), __uint_as_float(w[q + 1])};
      A[q] += fabsf(__uint_as_float(w[q]));
      A[q + 1] += fabsf(__uint_as_float(w[q + 1]));
    }
  };
  auto ld2 = [&](__amdgpu_buffer_rsrc_t rs, uint4 (&v)[2]) __attribute__((always_inline)) {
    const auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)voff, 0, 0);
    const auto b = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)voff + 16, 0, 0);
    v[0] = uint4{a[0], a[1], a[2], a[3]};
    v[1] = uint4{b[0], b[1], b[2], b[3]};
  };
  int jj = 0;
  for (; jj + BGU <= jn; jj += BGU) {
    uint4 v[BGU][2];
#pragma unroll
    for (int g = 0; g < BGU; ++g) ld2(row(jj + g), v[g]);
#pragma unroll
    for (int g = 0; g < BGU; ++g) acc(v[g]);
  }
  for (; jj < jn; ++jj) {
    uint4 v[2];
    ld2(row(jj), v);
    acc(v);
  }
}

__device__ __forceinline__ float sigmoid_ref(float l) { return 1.0f / (1.0f + expf(-l)); }
__device__ __forceinline__ unsigned long long score_key(float sc, int64_t c) {
  return ((unsigned long long)ord_f32_p(sc) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)c);
}
constexpr unsigned long long KEY_SCORE_MAX = 0xFFFFFFFF00000000ull;   // above every score's key

// The interval of one candidate's exact score from its truncated sums (see above). hl == 0: the
// exact score 0.5 (logit 0). Returns false when the sums do not bound it (a zero or overflowing
// S^, non-finite sums): the candidate is then refined whatever tau is.
struct Bounds {
  float slo, shi, nlo, nhi, dlo, dhi;
  bool ok;
};
__device__ __forceinline__ Bounds make_bounds(float S, float N, float A, int64_t hl, float beta) {
  Bounds b;
  const float g = (float)hl * 0x1p-23f + 0x1p-20f;
  const float tiny = (float)hl * 0x1p-126f;   // truncation below the normal range (absolute)
  b.slo = S * (1.f - 3.f * g);
  b.shi = S * (1.f + 0x1p-7f) * (1.f + 3.f * g) + tiny;
  const float rn = (0x1p-7f + 4.f * g) * A + tiny;
  b.nlo = N - rn;
  b.nhi = N + rn;
  if (beta == 0.5f) {
    b.dlo = sqrtf(b.slo);
    b.dhi = sqrtf(b.shi);
  } else {
    const float p0 = powf(b.slo, beta), p1 = powf(b.shi, beta);
    b.dlo = fminf(p0, p1);
    b.dhi = fmaxf(p0, p1);
  }
  b.ok = b.slo > 0.f && b.dlo > 0.f && __builtin_isfinite(b.dhi) && __builtin_isfinite(b.nlo) &&
         __builtin_isfinite(b.nhi);
  return b;
}
__device__ __forceinline__ float upper_score(const Bounds& b) {
  float l = b.nhi >= 0.f ? b.nhi / b.dlo : b.nhi / b.dhi;
  l += fabsf(l) * 0x1p-19f;
  return fminf(sigmoid_ref(l) * (1.f + 0x1p-20f), 1.0f);
}
__device__ __forceinline__ float lower_score(const Bounds& b) {
  float l = b.nlo >= 0.f ? b.nlo / b.dhi : b.nlo / b.dlo;
  l -= fabsf(l) * 0x1p-19f;
  return l >= 17.f ? 1.0f : sigmoid_ref(l) * (1.f - 0x1p-20f);
}

// A cheap test that a candidate cannot reach the list's k-th key: its upper logit (v_rcp / v_sqrt,
// widened by 2^-17 to cover them and the accurate path's own rounding) is below L, the logit under
// which the accurate upper score stays below the k-th key's score (lthr_of). beta == 0.5 only
// (else L = -inf: no pruning); NaN anywhere keeps the candidate.
__device__ __forceinline__ bool may_reach(float S, float N, float A, int64_t hl, float L) {
  const float g = (float)hl * 0x1p-23f + 0x1p-20f;
  const float tiny = (float)hl * 0x1p-126f;
  const float nhi = N + ((0x1p-7f + 4.f * g) * A + tiny);
  const float sd = nhi >= 0.f ? S * (1.f - 3.f * g) : S * (1.f + 0x1p-7f) * (1.f + 3.f * g) + tiny;
  float l = nhi * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(sd));
  l += fabsf(l) * 0x1p-17f;
  return !(l < L);
}
// L for may_reach from the k-th key's score ts: upper_score(l) <= sigmoid_fp32(l) (1 + 2^-20) <
// ts for every l < L = logit(ts (1 - 2^-18)) less a margin (ts = 1.0f: L ~ 12.5, below which the
// upper score is < 1.0f). -inf when there is no such bound (list not full, ts <= 0, NaN, beta).
__device__ __forceinline__ float lthr_of(unsigned long long thr, float beta) {
  if (thr == 0ull || beta != 0.5f) return -__builtin_inff();
  const float ts = unord_f32_p((uint32_t)(thr >> 32));
  if (!(ts > 0.f && ts <= 1.f)) return -__builtin_inff();
  const double p = (double)ts * (1.0 - 0x1p-18);
  double L = log(p / (1.0 - p));
  L -= 1e-6 * (1.0 + fabs(L));
  return (float)L;
}

// Sorts the wave's LDS keys L[0 .. n) descending (bitonic over the next power of two >= 64,
// padded with 0 keys; L must have room for it).
__device__ void wave_sort_desc(unsigned long long* L, int n) {
  const int lane = threadIdx.x & 63;
  int n2 = 64;
  while (n2 < n) n2 <<= 1;
  for (int i = n + lane; i < n2; i += 64) L[i] = 0ull;
  wave_lds_sync();
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = lane; i < n2; i += 64) {
        const int partner = i ^ stride;
        if (partner > i) {
          const bool desc = (i & size) == 0;
          const unsigned long long a = L[i], b = L[partner];
          if (desc ? (a < b) : (a > b)) {
            L[i] = b;
            L[partner] = a;
          }
        }
      }
      wave_lds_sync();
    }
  }
}

// Merges the keys kq[q] with bit q of `offer` set (this lane's) into the wave's descending list
// L[0 .. cnt) in LDS; L has room for the padded power of two of cnt + offered. Returns the new
// count min(cnt + offered, k); L[0 .. that) is the new list.
template <int NQ>
__device__ int wave_merge_keys(unsigned long long* L, int cnt, const unsigned long long (&kq)[NQ],
                               uint32_t offer, int k) {
  const int lane = threadIdx.x & 63;
  const int mine_n = __popc(offer);
  int excl = mine_n;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(excl, o);
    if (lane >= o) excl += y;
  }
  const int m = __shfl(excl, 63);
  excl -= mine_n;
  if (m == 0) return cnt;
  int pos = cnt + excl;
#pragma unroll
  for (int q = 0; q < NQ; ++q)
    if ((offer >> q) & 1u) L[pos++] = kq[q];
  const int n = cnt + m;
  wave_sort_desc(L, n);
  return n < k ? n : k;
}

__global__ void __launch_bounds__(GW * 64)
pair_bound_topk_kernel(const uint32_t* __restrict__ HI, int64_t ld, const int32_t* __restrict__ rowmap,
                       const int64_t* __restrict__ indptr, const int64_t* __restrict__ indices,
                       const int32_t* __restrict__ users, int32_t nusers, int64_t col0, int64_t cols,
                       float beta, int k, unsigned long long* __restrict__ lokeys,
                       int32_t* __restrict__ locount, unsigned long long* __restrict__ surv,
                       int32_t* __restrict__ scount, int cap, const int32_t* __restrict__ erows,
                       const int64_t* __restrict__ spans, int32_t* __restrict__ work) {
  __shared__ unsigned long long lk[GW][BK_LDS];
  __shared__ uint32_t hm[GW][BSTRIPE / 32];   // history POIs of this block, one bit per column
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int GQ = 4;
  int64_t qnext = 0, qend = 0;
  for (int64_t it = 0;; ++it) {
  int64_t slot;
  if (work) {
    if (qnext == qend) {
      int got = 0;
      if (lane == 0) got = atomicAdd(work, GQ);
      qnext = __builtin_amdgcn_readfirstlane(got);
      qend = qnext + GQ;
    }
    slot = qnext++;
  } else {
    if (it > 0) break;
    slot = int64_t(blockIdx.x) * GW + w;
  }
  if (slot >= nusers) break;                 // wave-uniform; no workgroup barriers below
  // the slot's history span: one load with spans (else users[slot] -> indptr, two in a row)
  int64_t hb, hl;
  if (spans) {
    hb = spans[2 * slot];
    hl = spans[2 * slot + 1];
  } else {
    const int64_t u = users[slot];
    hb = indptr[u];
    hl = indptr[u + 1] - hb;
  }
  // the slot's list state, loaded before the gather (independent of it): its latency overlaps
  // the row reads instead of following them
  const int cnt = locount[slot];
  const unsigned long long lk_last = lokeys[slot * k + k - 1];   // meaningful when cnt == k
  int sc = scount[slot];
  const int64_t x = int64_t(lane) * BCPL;    // column within the block [col0, col0 + cols)
  if (lane < BSTRIPE / 32) hm[w][lane] = 0u;
  wave_lds_sync();
  f2v S2[BCPL / 2], N2[BCPL / 2];
  float A[BCPL];
#pragma unroll
  for (int q = 0; q < BCPL / 2; ++q) S2[q] = N2[q] = f2v{0.f, 0.f};
#pragma unroll
  for (int q = 0; q < BCPL; ++q) A[q] = 0.f;
  for (int64_t j0 = 0; j0 < hl; j0 += 64) {
    const int jn = __builtin_amdgcn_readfirstlane((int)std::min<int64_t>(64, hl - j0));
    int32_t mrow = 0;
    if (lane < jn) {
      // with erows the entry's table row loads beside its POI id (else rowmap[id], after it)
      const int64_t e = hb + j0 + lane;
      const int64_t c = indices[e];
      mrow = erows ? erows[e] : rowmap[c];
      const int64_t r = c - col0;
      if (r >= 0 && r < cols) atomicOr(&hm[w][r >> 5], 1u << (r & 31));
    }
    bound_rows(HI, ld, mrow, jn, (uint32_t)(cols * 4), (uint32_t)(x * 4), S2, N2, A);
  }
  wave_lds_sync();
  float S[BCPL], N[BCPL];
#pragma unroll
  for (int q = 0; q < BCPL; ++q) {
    S[q] = S2[q / 2][q & 1];
    N[q] = N2[q / 2][q & 1];
  }
  const unsigned long long thr = cnt == k ? lk_last : 0ull;   // valid keys are > 0
  // upper keys of every candidate; lower keys only where the upper one reaches thr (else neither
  // can enter the list nor survive). Held as their score halves (the id half is the column's), so
  // the epilogue does not outgrow the gather loop's registers.
  uint32_t ho[BCPL], lo_[BCPL];
  uint32_t live = 0, offer = 0;
  const uint32_t idb0 = 0xFFFFFFFFu - (uint32_t)(col0 + x);   // id half of column x; x + q: - q
  auto key_of = [&](uint32_t ord, int q) __attribute__((always_inline)) {
    return ((unsigned long long)ord << 32) | (unsigned long long)(idb0 - (uint32_t)q);
  };
  const float Lthr = lthr_of(thr, beta);   // wave-uniform
#pragma unroll
  for (int q = 0; q < BCPL; ++q) {
    ho[q] = 0u;
    lo_[q] = 0u;
    const int64_t r = x + q;
    if (r < cols && !((hm[w][r >> 5] >> (r & 31)) & 1u)) {
      if (hl == 0) {   // exact: logit 0 -> 0.5 for every candidate
        live |= 1u << q;
        ho[q] = lo_[q] = ord_f32_p(0.5f);
      } else if (may_reach(S[q], N[q], A[q], hl, Lthr)) {
        live |= 1u << q;
        const Bounds b = make_bounds(S[q], N[q], A[q], hl, beta);
        ho[q] = b.ok ? ord_f32_p(upper_score(b)) : 0xFFFFFFFFu;
        if (b.ok && key_of(ho[q], q) > thr) lo_[q] = ord_f32_p(lower_score(b));
      }
      if (lo_[q] != 0u && key_of(lo_[q], q) > thr) offer |= 1u << q;
    }
  }
  // the list of lower bounds: two merges of <= 256 offered keys (the LDS holds k + 256)
  unsigned long long* L = lk[w];
  int nk = cnt;
  const bool merged = __ballot(offer != 0u) != 0ull;
  if (merged) {
    for (int i = lane; i < cnt; i += 64) L[i] = lokeys[slot * k + i];
    wave_lds_sync();
    const unsigned long long l0[4] = {key_of(lo_[0], 0), key_of(lo_[1], 1), key_of(lo_[2], 2), key_of(lo_[3], 3)};
    const unsigned long long l1[4] = {key_of(lo_[4], 4), key_of(lo_[5], 5), key_of(lo_[6], 6), key_of(lo_[7], 7)};
    nk = wave_merge_keys<4>(L, nk, l0, offer & 0xFu, k);
    nk = wave_merge_keys<4>(L, nk, l1, offer >> 4, k);
    for (int i = lane; i < nk; i += 64) lokeys[slot * k + i] = L[i];
    if (lane == 0) locount[slot] = nk;
  }
  const unsigned long long tau = nk == k ? (merged ? L[k - 1] : thr) : 0ull;
  // survivors: upper key >= tau, appended to the user's list
  uint32_t sv = 0;
#pragma unroll
  for (int q = 0; q < BCPL; ++q)
    if (((live >> q) & 1u) && key_of(ho[q], q) >= tau) sv |= 1u << q;
  const int mine_n = __popc(sv);
  int excl = mine_n;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(excl, o);
    if (lane >= o) excl += y;
  }
  const int m = __shfl(excl, 63);
  excl -= mine_n;
  if (m > 0 && sc >= 0) {
    unsigned long long* list = surv + slot * (int64_t)cap;
    if (sc + m > cap) {   // compact by the current tau (in place: a write never passes the chunk read)
      int wpos = 0;
      for (int i0 = 0; i0 < sc; i0 += 64) {
        const bool in = i0 + lane < sc;
        const unsigned long long v = in ? list[i0 + lane] : 0ull;
        const bool keep = in && v >= tau;
        const unsigned long long bal = __ballot(keep);
        const int before = __popcll(bal & ((1ull << lane) - 1ull));
        if (keep) list[wpos + before] = v;
        wpos += __popcll(bal);
      }
      sc = wpos + m > cap ? -1 : wpos;   // -1: overflow, refined over the whole column range
    }
    if (sc >= 0) {
      int pos = sc + excl;
#pragma unroll
      for (int q = 0; q < BCPL; ++q)
        if ((sv >> q) & 1u) list[pos++] = key_of(ho[q], q);
      sc += m;
    }
    if (lane == 0) scount[slot] = sc;
  }
  wave_lds_sync();   // the next slot's hm / lk writers after this slot's readers
  }
}

// Phase 2: per user, the exact scores of the candidates whose upper key reaches the final tau (all
// columns of [col0, col0 + cols) for an overflowed user), from the ex pairs of the block tables
//   X + b * bstride + row * ld + x  (uint2 pairs),  column col0 + b * bcols + x,
// summed in history (CSR) order as pair_gather_topk_kernel sums them, 64 candidates (one per lane)
// at a time; a running top-k in LDS. stats[0] += candidates refined, stats[1] += overflowed users.
constexpr int RF_LDS = 512;   // running list (k <= 256) + 64 offered, padded to a power of two
constexpr int RF_CAND = 512;  // kept survivors sorted in LDS (more: streamed unsorted)

__global__ void __launch_bounds__(GW * 64)
pair_refine_topk_kernel(const uint2* __restrict__ X, int64_t bstride, int64_t ld,
                        int64_t bcols, const int32_t* __restrict__ rowmap,
                        const int64_t* __restrict__ indptr, const int64_t* __restrict__ indices,
                        const int32_t* __restrict__ users, int32_t nusers, int64_t col0, int64_t cols,
                        float beta, int k, const unsigned long long* __restrict__ lokeys,
                        const int32_t* __restrict__ locount, const unsigned long long* __restrict__ surv,
                        const int32_t* __restrict__ scount, int cap,
                        const unsigned long long* __restrict__ tau_in, unsigned long long* __restrict__ keys,
                        int32_t* __restrict__ kcount, int32_t* __restrict__ nan_count,
                        int32_t* __restrict__ stats, const int32_t* __restrict__ erows) {
  __shared__ unsigned long long lk[GW][RF_LDS];
  __shared__ uint32_t cb[GW][128];   // pending candidate columns (relative to col0)
  __shared__ unsigned long long ck[GW][RF_CAND];   // kept survivors' upper keys, sorted
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t slot = int64_t(blockIdx.x) * GW + w;
  if (slot >= nusers) return;                // wave-uniform; no workgroup barriers below
  const int64_t u = users[slot];
  const int64_t hb = indptr[u], hl = indptr[u + 1] - hb;
  const int cnt = locount[slot];
  // tau_in: a threshold at least this large, e.g. the k-th lower key over every column shard of a
  // process group (each shard then refines only what can reach the GLOBAL top-k)
  unsigned long long tau = cnt == k ? lokeys[slot * k + k - 1] : 0ull;
  if (tau_in && tau_in[slot] > tau) tau = tau_in[slot];
  const int sc = scount[slot];
  unsigned long long* L = lk[w];
  int nk = 0;             // the running exact list L[0 .. nk)
  int nan = 0, refined = 0;
  // exact keys of the columns r (valid lanes) -> merged into L
  auto batch = [&](int64_t r, bool valid) __attribute__((always_inline)) {
    const int64_t rr = valid ? r : 0;                   // invalid lanes read a column that exists
    const int64_t b = rr / bcols;
    const int64_t xo = b * bstride + (rr - b * bcols);  // in (e, e*s) pairs
    const int64_t c = col0 + rr;
    float Sa = 0.f, Na = 0.f;
    bool in_hist = false;
    for (int64_t j0 = 0; j0 < hl; j0 += 64) {
      const int jn = __builtin_amdgcn_readfirstlane((int)std::min<int64_t>(64, hl - j0));
      int64_t mine = 0, mid = -1;
      if (lane < jn) {
        mid = indices[hb + j0 + lane];
        mine = int64_t(erows ? erows[hb + j0 + lane] : rowmap[mid]) * ld;   // ex rows hold ld pairs
      }
      const uint32_t mlo = uint32_t(mine), mhi = uint32_t(mine >> 32);
      const uint32_t ilo = uint32_t(mid), ihi = uint32_t(mid >> 32);
      int jj = 0;
      for (; jj + GU <= jn; jj += GU) {
        uint2 v[GU];
        int64_t id[GU];
#pragma unroll
        for (int g = 0; g < GU; ++g) {
          id[g] = bcast64(ilo, ihi, jj + g);
          v[g] = X[bcast64(mlo, mhi, jj + g) + xo];   // one 8-byte read: one line per pair
        }
#pragma unroll
        for (int g = 0; g < GU; ++g) {
          Sa += __uint_as_float(v[g].x);
          Na += __uint_as_float(v[g].y);
          in_hist |= id[g] == c;
        }
      }
      for (; jj < jn; ++jj) {
        const uint2 v = X[bcast64(mlo, mhi, jj) + xo];
        Sa += __uint_as_float(v.x);
        Na += __uint_as_float(v.y);
        in_hist |= bcast64(ilo, ihi, jj) == c;
      }
    }
    unsigned long long kq[1] = {0ull};
    uint32_t offer = 0;
    if (valid && !in_hist) {
      float logit = 0.f;   // empty history: logit 0
      if (hl > 0) logit = Na / ((beta == 0.5f) ? sqrtf(Sa) : powf(Sa, beta));
      float s = 1.0f / (1.0f + expf(-logit));
      if (logit != logit) {
        s = __builtin_nanf("");
        ++nan;
      }
      kq[0] = score_key(s, c);
      ++refined;
      const unsigned long long lthr = nk == k ? L[k - 1] : 0ull;
      if (kq[0] > lthr) offer = 1u;
    }
    wave_lds_sync();
    nk = wave_merge_keys<1>(L, nk, kq, offer, k);
  };
  if (sc < 0) {   // overflowed: every column of the range
    for (int64_t r0 = 0; r0 < cols; r0 += 64) batch(r0 + lane, r0 + lane < cols);
  } else {
    const unsigned long long* list = surv + slot * (int64_t)cap;
    // the kept survivors (upper key >= tau), sorted by upper key when they fit the LDS: refined in
    // that order, 64 at a time, until the list's k-th exact key is above the next one's upper key
    // (no candidate after it can enter) -- ~64 instead of ~84 per user at config 4
    unsigned long long* C = ck[w];
    int nkept = 0;
    for (int i0 = 0; i0 < sc; i0 += 64) {
      const bool in = i0 + lane < sc;
      const unsigned long long v = in ? list[i0 + lane] : 0ull;
      const bool keep = in && v >= tau;
      const unsigned long long bal = __ballot(keep);
      const int pos = nkept + __popcll(bal & ((1ull << lane) - 1ull));
      if (keep && pos < RF_CAND) C[pos] = v;
      nkept += __popcll(bal);
    }
    if (nkept <= RF_CAND) {
      wave_sort_desc(C, nkept);
      for (int b0 = 0; b0 < nkept; b0 += 64) {
        if (nk == k && L[k - 1] > C[b0]) break;   // wave-uniform (LDS, synced by the merge)
        const bool in = b0 + lane < nkept;
        const unsigned long long v = in ? C[b0 + lane] : 0ull;
        batch((int64_t)((0xFFFFFFFFu - (uint32_t)(v & 0xFFFFFFFFull)) - (uint32_t)col0), in);
      }
      nkept = -1;   // done
    }
    int pend = 0;   // cb[w][0 .. pend)
    for (int i0 = 0; nkept >= 0 && i0 < sc; i0 += 64) {
      const bool in = i0 + lane < sc;
      const unsigned long long v = in ? list[i0 + lane] : 0ull;
      const bool keep = in && v >= tau;
      const unsigned long long bal = __ballot(keep);
      if (keep) cb[w][pend + __popcll(bal & ((1ull << lane) - 1ull))] =
          (uint32_t)((0xFFFFFFFFu - (uint32_t)(v & 0xFFFFFFFFull)) - (uint32_t)col0);
      pend += __popcll(bal);
      wave_lds_sync();
      if (pend >= 64) {
        const uint32_t r = cb[w][lane];
        const uint32_t rest = lane < pend - 64 ? cb[w][64 + lane] : 0u;
        wave_lds_sync();
        if (lane < pend - 64) cb[w][lane] = rest;
        pend -= 64;
        wave_lds_sync();
        batch((int64_t)r, true);
      }
    }
    if (nkept >= 0 && pend > 0) {
      const uint32_t r = lane < pend ? cb[w][lane] : 0u;
      batch((int64_t)r, lane < pend);
    }
  }
  for (int i = lane; i < nk; i += 64) keys[slot * k + i] = L[i];
  if (lane == 0) kcount[slot] = nk;
  if (nan_count) {
    for (int o = 32; o > 0; o >>= 1) nan += __shfl_xor(nan, o);
    if (lane == 0 && nan) atomicAdd(nan_count, nan);
  }
  if (stats) {
    for (int o = 32; o > 0; o >>= 1) refined += __shfl_xor(refined, o);
    if (lane == 0) {
      atomicAdd(stats, refined);
      if (sc < 0) atomicAdd(stats + 1, 1);
    }
  }
}

// keys -> (ids, scores) of the top-k lists; short lists padded with -1 / NaN and counted
__global__ void topk_keys_finish_kernel(const unsigned long long* __restrict__ keys,
                                        const int32_t* __restrict__ kcount, int32_t n, int k,
                                        int32_t* __restrict__ out_ids, float* __restrict__ out_scores,
                                        int32_t* __restrict__ short_count) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= int64_t(n) * k) return;
  const int64_t slot = i / k;
  const int r = int(i % k);
  const int cnt = kcount[slot];
  int32_t id = -1;
  float sc = __builtin_nanf("");
  if (r < cnt) {
    const unsigned long long key = keys[i];
    id = (int32_t)(0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull));
    sc = unord_f32_p((uint32_t)(key >> 32));
  }
  out_ids[i] = id;
  out_scores[i] = sc;
  if (r == 0 && cnt < k && short_count) atomicAdd(short_count, 1);
}

}  // namespace

extern "C" {

size_t nais_pair_rows_workspace_size(int64_t num_pois) {
  if (num_pois <= 0) return 0;
  return size_t((num_pois + SCAN_THREADS - 1) / SCAN_THREADS) * sizeof(int32_t);
}

int32_t nais_pair_rows(const int64_t* indptr, const int64_t* indices, const int32_t* users,
                       int32_t num_users, int64_t num_pois, int32_t* rowmap, int64_t* items,
                       int64_t* num_items, void* workspace, size_t workspace_bytes, void* stream) {
  if (num_users < 0 || num_pois <= 0) return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (!rowmap || !items || !num_items || (num_users > 0 && (!indptr || !indices || !users)))
    return nais_internal_fail(NAIS_E_INVALID, "missing pointer");
  if (!workspace || workspace_bytes < nais_pair_rows_workspace_size(num_pois))
    return nais_internal_fail(NAIS_E_WORKSPACE, "workspace too small (nais_pair_rows_workspace_size)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(rowmap, 0, size_t(num_pois) * sizeof(int32_t), st) != hipSuccess)
    return nais_internal_fail(NAIS_E_HIP, "memset failed");
  for (int32_t u0 = 0; u0 < num_users; u0 += 65535) {
    const int nb = std::min<int32_t>(65535, num_users - u0);
    hipLaunchKernelGGL(mark_kernel, dim3((unsigned)nb), dim3(256), 0, st, indptr, indices, users + u0,
                       rowmap);
  }
  const int64_t nb = (num_pois + SCAN_THREADS - 1) / SCAN_THREADS;
  int32_t* bsum = static_cast<int32_t*>(workspace);
  hipLaunchKernelGGL(count_kernel, dim3((unsigned)nb), dim3(SCAN_THREADS), 0, st, rowmap, num_pois, bsum);
  hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(SCAN_THREADS), 0, st, bsum, nb, num_items);
  hipLaunchKernelGGL(place_kernel, dim3((unsigned)nb), dim3(SCAN_THREADS), 0, st, rowmap, num_pois,
                     bsum, items);
  return nais_internal_check_launch("pair rows");
}

int32_t nais_pair_gather(const float* e, const float* es, int64_t ld, const int32_t* rowmap,
                         const int64_t* indptr, const int64_t* indices, const int32_t* users,
                         int32_t num_users, int64_t col0, int64_t cols, float beta, float* scores,
                         int64_t score_ld, int64_t score_col0, int32_t* nan_count, void* stream) {
  if (num_users < 0 || col0 < 0 || cols < 0 || ld < cols || col0 < score_col0 ||
      score_ld < col0 - score_col0 + cols)
    return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (num_users == 0 || cols == 0) return NAIS_OK;
  if (!e || !es || !rowmap || !indptr || !indices || !users || !scores)
    return nais_internal_fail(NAIS_E_INVALID, "missing pointer");
  if (ld % 4 != 0) return nais_internal_fail(NAIS_E_INVALID, "ld must be a multiple of 4");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t stripes = (cols + STRIPE - 1) / STRIPE;
  if (stripes > 65535) return nais_internal_fail(NAIS_E_UNSUPPORTED, "cols > 65535 * 256");
  hipLaunchKernelGGL(pair_gather_kernel, dim3((unsigned)((num_users + GW - 1) / GW), (unsigned)stripes),
                     dim3(GW * 64), 0, st, e, es, ld, rowmap, indptr, indices, users, num_users, col0,
                     cols, beta, scores, score_ld, score_col0, nan_count);
  return nais_internal_check_launch("pair_gather_kernel");
}

int32_t nais_pair_gather_topk(const float* e, const float* es, int64_t ld, const int32_t* rowmap,
                              const int64_t* indptr, const int64_t* indices, const int32_t* users,
                              int32_t num_users, int64_t col0, int64_t cols, float beta, int32_t k,
                              uint64_t* keys, int32_t* kcount, int32_t* nan_count, int32_t* work,
                              void* stream) {
  if (num_users < 0 || col0 < 0 || cols < 0 || ld < cols || k <= 0)
    return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (k > TK_LDS - STRIPE) return nais_internal_fail(NAIS_E_UNSUPPORTED, "k must be <= 256");
  if (col0 + cols > 0xFFFFFFFFll) return nais_internal_fail(NAIS_E_UNSUPPORTED, "POI ids must fit 32 bits");
  if (num_users == 0 || cols == 0) return NAIS_OK;
  if (!e || !es || !rowmap || !indptr || !indices || !users || !keys || !kcount)
    return nais_internal_fail(NAIS_E_INVALID, "missing pointer");
  if (ld % 4 != 0) return nais_internal_fail(NAIS_E_INVALID, "ld must be a multiple of 4");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  unsigned groups = (unsigned)((num_users + GW - 1) / GW);
  if (work) {   // a work queue: one resident round of workgroups on the stream's CUs (5 per CU)
    const int ncu = nais_internal_stream_cus(st);
    if (ncu <= 0) return nais_internal_fail(NAIS_E_HIP, "device attributes");
    groups = std::min<unsigned>(groups, (unsigned)ncu * 5u);
  }
  for (int64_t s0 = 0; s0 < cols; s0 += STRIPE) {   // one launch per stripe: one writer per list
    if (work && hipMemsetAsync(work, 0, sizeof(int32_t), st) != hipSuccess)
      return nais_internal_fail(NAIS_E_HIP, "hipMemsetAsync(work)");
    hipLaunchKernelGGL(pair_gather_topk_kernel, dim3(groups), dim3(GW * 64), 0, st, e + s0, es + s0, ld,
                       rowmap, indptr, indices, users, num_users, col0 + s0,
                       std::min<int64_t>(STRIPE, cols - s0), beta, (int)k,
                       reinterpret_cast<unsigned long long*>(keys), kcount, nan_count, work);
    const int32_t rc = nais_internal_check_launch("pair_gather_topk_kernel");
    if (rc) return rc;
  }
  return NAIS_OK;
}

int32_t nais_pair_bound_topk(const uint32_t* hi, int64_t ld, const int32_t* rowmap,
                             const int64_t* indptr, const int64_t* indices, const int32_t* users,
                             int32_t num_users, int64_t col0, int64_t cols, float beta, int32_t k,
                             uint64_t* lo_keys, int32_t* lo_count, uint64_t* surv, int32_t* surv_count,
                             int32_t surv_cap, const int32_t* entry_rows, const int64_t* spans,
                             int32_t* work, void* stream) {
  if (num_users < 0 || col0 < 0 || cols < 0 || ld < cols || k <= 0 || surv_cap < 64)
    return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (k > BK_LDS - 256) return nais_internal_fail(NAIS_E_UNSUPPORTED, "k must be <= 256");
  if (col0 + cols > 0xFFFFFFFFll) return nais_internal_fail(NAIS_E_UNSUPPORTED, "POI ids must fit 32 bits");
  if (num_users == 0 || cols == 0) return NAIS_OK;
  if (!hi || !rowmap || !indptr || !indices || !users || !lo_keys || !lo_count || !surv || !surv_count)
    return nais_internal_fail(NAIS_E_INVALID, "missing pointer");
  if (ld % 4 != 0 || (reinterpret_cast<uintptr_t>(hi) & 15) != 0)
    return nais_internal_fail(NAIS_E_INVALID, "ld must be a multiple of 4 and hi 16-byte aligned");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  unsigned groups = (unsigned)((num_users + GW - 1) / GW);
  if (work) {   // a work queue: one resident round of workgroups on the stream's CUs (5 per CU)
    const int ncu = nais_internal_stream_cus(st);
    if (ncu <= 0) return nais_internal_fail(NAIS_E_HIP, "device attributes");
    groups = std::min<unsigned>(groups, (unsigned)ncu * 5u);
  }
  for (int64_t s0 = 0; s0 < cols; s0 += BSTRIPE) {   // one launch per stripe: one writer per list
    if (work && hipMemsetAsync(work, 0, sizeof(int32_t), st) != hipSuccess)
      return nais_internal_fail(NAIS_E_HIP, "hipMemsetAsync(work)");
    hipLaunchKernelGGL(pair_bound_topk_kernel, dim3(groups), dim3(GW * 64), 0, st, hi + s0, ld, rowmap,
                       indptr, indices, users, num_users, col0 + s0, std::min<int64_t>(BSTRIPE, cols - s0),
                       beta, (int)k, reinterpret_cast<unsigned long long*>(lo_keys), lo_count,
                       reinterpret_cast<unsigned long long*>(surv), surv_count, (int)surv_cap, entry_rows,
                       spans, work);
    const int32_t rc = nais_internal_check_launch("pair_bound_topk_kernel");
    if (rc) return rc;
  }
  return NAIS_OK;
}

int32_t nais_pair_refine_topk(const uint32_t* ex, int64_t block_stride,
                              int64_t ld, int64_t block_cols, const int32_t* rowmap,
                              const int64_t* indptr, const int64_t* indices, const int32_t* users,
                              int32_t num_users, int64_t col0, int64_t cols, float beta, int32_t k,
                              const uint64_t* lo_keys, const int32_t* lo_count, const uint64_t* surv,
                              const int32_t* surv_count, int32_t surv_cap, const uint64_t* tau,
                              uint64_t* keys, int32_t* kcount, int32_t* nan_count, int32_t* stats,
                              const int32_t* entry_rows, void* stream) {
  if (num_users < 0 || col0 < 0 || cols < 0 || k <= 0 || surv_cap < 64 || block_cols <= 0 ||
      ld < std::min<int64_t>(block_cols, cols) || block_stride < 0 || block_stride % 2 != 0)
    return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (k > RF_LDS - 256) return nais_internal_fail(NAIS_E_UNSUPPORTED, "k must be <= 256");
  if (col0 + cols > 0xFFFFFFFFll) return nais_internal_fail(NAIS_E_UNSUPPORTED, "POI ids must fit 32 bits");
  if (num_users == 0) return NAIS_OK;
  if (!rowmap || !indptr || !indices || !users || !lo_keys || !lo_count || !surv || !surv_count ||
      !keys || !kcount || (cols > 0 && !ex))
    return nais_internal_fail(NAIS_E_INVALID, "missing pointer");
  hipLaunchKernelGGL(pair_refine_topk_kernel, dim3((unsigned)((num_users + GW - 1) / GW)), dim3(GW * 64), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const uint2*>(ex), block_stride / 2, ld,
                     block_cols,
                     rowmap, indptr, indices, users, num_users, col0, cols, beta, (int)k,
                     reinterpret_cast<const unsigned long long*>(lo_keys), lo_count,
                     reinterpret_cast<const unsigned long long*>(surv), surv_count, (int)surv_cap,
                     reinterpret_cast<const unsigned long long*>(tau),
                     reinterpret_cast<unsigned long long*>(keys), kcount, nan_count, stats, entry_rows);
  return nais_internal_check_launch("pair_refine_topk_kernel");
}

int32_t nais_pair_prior_table(const double* coords, int64_t num_pois, const int64_t* items,
                              int64_t num_items, int64_t col0, int64_t cols, double a, double b,
                              double* pr, int64_t ld, void* stream) {
  if (num_pois <= 0 || num_items < 0 || col0 < 0 || cols < 0 || col0 + cols > num_pois || ld < cols)
    return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (num_items == 0 || cols == 0) return NAIS_OK;
  if (!coords || !items || !pr) return nais_internal_fail(NAIS_E_INVALID, "missing pointer");
  const int64_t gy = (num_items + 15) / 16;
  if (gy > 65535ll * 1024) return nais_internal_fail(NAIS_E_UNSUPPORTED, "too many items");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int64_t y0 = 0; y0 < gy; y0 += 65535) {
    const int64_t ny = std::min<int64_t>(65535, gy - y0);
    hipLaunchKernelGGL(prior_pair_table_kernel,
                       dim3((unsigned)((cols + PRIOR_TAB_THREADS - 1) / PRIOR_TAB_THREADS), (unsigned)ny),
                       dim3(PRIOR_TAB_THREADS), 0, st, coords, items + y0 * 16,
                       std::min<int64_t>(num_items - y0 * 16, ny * 16), col0, cols, a, b,
                       pr + y0 * 16 * ld, ld);
    const int32_t rc = nais_internal_check_launch("prior_pair_table_kernel");
    if (rc) return rc;
  }
  return NAIS_OK;
}

int32_t nais_pair_prior_gather(const double* pr, int64_t ld, const int32_t* rowmap,
                               const int64_t* indptr, const int64_t* indices, const int32_t* users,
                               int32_t num_users, int64_t col0, int64_t cols, double* g, int64_t g_ld,
                               int64_t g_col0, uint64_t* gmax_bits, int32_t flags, void* stream) {
  if (num_users < 0 || col0 < 0 || cols < 0 || ld < cols || col0 < g_col0 || g_ld < col0 - g_col0 + cols)
    return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (num_users == 0 || cols == 0) return NAIS_OK;
  if (!pr || !rowmap || !indptr || !indices || !users || !g || !gmax_bits)
    return nais_internal_fail(NAIS_E_INVALID, "missing pointer");
  if (ld % 4 != 0) return nais_internal_fail(NAIS_E_INVALID, "ld must be a multiple of 4 (32-byte loads)");
  const int64_t stripes = (cols + STRIPE - 1) / STRIPE;
  if (stripes > 65535) return nais_internal_fail(NAIS_E_UNSUPPORTED, "cols > 65535 * 256");
  hipLaunchKernelGGL(prior_pair_gather_kernel,
                     dim3((unsigned)((num_users + GW - 1) / GW), (unsigned)stripes), dim3(GW * 64), 0,
                     reinterpret_cast<hipStream_t>(stream), pr, ld, rowmap, indptr, indices, users,
                     num_users, col0, cols, g, g_ld, g_col0,
                     reinterpret_cast<unsigned long long*>(gmax_bits),
                     (flags & NAIS_PRIOR_FINITE) ? 1 : 0);
  return nais_internal_check_launch("prior_pair_gather_kernel");
}

int32_t nais_topk_keys_finish(const uint64_t* keys, const int32_t* kcount, int32_t num_users, int32_t k,
                              int32_t* out_ids, float* out_scores, int32_t* short_count, void* stream) {
  if (num_users < 0 || k <= 0) return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (num_users == 0) return NAIS_OK;
  if (!keys || !kcount || !out_ids || !out_scores) return nais_internal_fail(NAIS_E_INVALID, "missing pointer");
  const int64_t total = int64_t(num_users) * k;
  hipLaunchKernelGGL(topk_keys_finish_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const unsigned long long*>(keys),
                     kcount, num_users, (int)k, out_ids, out_scores, short_count);
  return nais_internal_check_launch("topk_keys_finish_kernel");
}

int32_t nais_stream_create_cu_mask(const uint32_t* cu_mask, uint32_t mask_words, void** stream) {
  if (!cu_mask || !mask_words || !stream) return nais_internal_fail(NAIS_E_INVALID, "bad arguments");
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, mask_words, cu_mask);
  if (e != hipSuccess)
    return nais_internal_fail(NAIS_E_HIP, (std::string("hipExtStreamCreateWithCUMask: ") +
                                           hipGetErrorString(e)).c_str());
  *stream = s;
  return NAIS_OK;
}

int32_t nais_stream_destroy(void* stream) {
  if (!stream) return NAIS_OK;
  return hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)) == hipSuccess
             ? NAIS_OK
             : nais_internal_fail(NAIS_E_HIP, "hipStreamDestroy failed");
}

}  // extern "C"
