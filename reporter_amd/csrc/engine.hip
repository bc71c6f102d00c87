// engine.hip — gfx950 kernels of the batched map matcher and their host driver.
//
// Replaces the work done inside valhalla.SegmentMatcher().Match (reference
// py/reporter_service.py:240, py/simple_reporter.py:166): meili's candidate
// search, transition routing, Viterbi and OSMLR segment forming, then the
// reference's own post-match report() (py/reporter_service.py:79-179).
//
// Stage / kernel map (DESIGN.md §5 has the rooflines):
//   k_states          one wave per trace: interpolation rule -> state layers
//   k_loc_*           locality order (large graphs): state slots counted into 64 x 64 Morton regions
//   k_candidates_lane K1, one lane per state: cell-major 32-byte records, per-road minima in
//                     registers, top 16 by (sq, road); k_candidates_wave takes the overflow
//   k_trans_count     pair constants + counts; k_scan_* lay out routes and K2 items
//   k_routes_ball2    K2, block-expanded: one lane per transition, two route-ball probes per
//                     target; search tiers (lane / reg2 / wave LDS / global) for the hand-overs
//   k_viterbi         K3, one 16-lane DPP row per trace: fp64 costs in registers, backtrace
//   k_paths_ball      one lane per chosen transition: labels from the balls, walk back by the
//                     rows' canonical predecessors (+ the search tiers)
//   k_rec_slot / k_seg_wave   K4: one wave per trace, traversal records 64 per step, runs by ballot
//   k_report          A8 epilogue, one wave per trace: report() + speed histogram + duration sums
//
// All arithmetic follows rm_common.hpp; compiled with -ffp-contract=off so the
// results are bit-identical to oracle/meili_oracle.c.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <type_traits>

#include "engine.hpp"
#include "json_points.hpp"

namespace rm {

const char* const kKernelNames[kNumKernels] = {"states", "candidates", "scan", "routes",
                                               "viterbi", "paths", "segments", "report", "locality"};

namespace {

constexpr uint32_t kEmpty = 0xffffffffu;
constexpr int kWave = 64;
constexpr int kBigH = 4096;     // LDS hash slots, retry tier (one source at a time)
constexpr int kMidH = 512;      // LDS hash slots, first wave tier
constexpr uint32_t kMidGrid = 4096;   // blocks of the 512-slot wave tiers (16 per CU)
constexpr int kCandH = 256;     // road hash slots in the candidate kernel
constexpr int kInlinePath = 8;  // path edges stored inline per slot (no allocation)
constexpr int kReg2Grid = 512;  // blocks of the second register tiers (grid-stride over their work lists)
constexpr uint32_t kMaxBoundCm = 100000000u;
constexpr double kQueueSpeedMps = 2.7777777777777777;  // 10 km/h

struct DevBatch {  // POD view of the workspace for kernels
  uint32_t T;
  uint64_t P;
  const uint32_t* trace_off; const float* lon; const float* lat; const double* time; const float* acc;
  const MatchOptions* opts; const uint32_t* trace_opt;
  uint32_t* slot_trace; uint32_t* n_states; uint32_t* state_orig; double* state_time;
  uint8_t* cand_n; uint4* cand_desc; float* cand_sq;
  uint32_t* trans_cnt; uint32_t* trans_off; double* gc; uint32_t* route; uint4* pair_info;
  // per transition with turn costs (rule 3b): the distance term K3 adds, turn_m + |route_m - gc| in
  // metres (+inf for an invalid route); null when no trace of the batch has turn costs
  double* route_d;
  uint32_t* walk;   // turn weights K2 leaves to k_turn_walks: per K2 block a count and its entries
  uint32_t* src_cnt; uint32_t* src_off; uint32_t* src_item;  // (pair, source) work items of K2
  int8_t* choice; uint8_t* chain_start; uint8_t* bp;
  uint32_t* path_off; uint32_t* path_cnt; uint32_t* path_inline; uint32_t* path_pool; uint64_t path_cap; uint32_t* route_dist;
  uint2* path_sab;   // per chosen transition: offsets (cm) of its source and target candidates on their roads
  SegmentRec* segs; uint32_t* seg_base; uint32_t* seg_cnt;
  uint32_t* trav_off;
  ReportRec* reps; uint32_t* rep_cnt; ReportStats* stats;
  // control words: [0] path pool used [2] error flags [3] routes list A [4] paths list A
  // [5] routes list B [6] paths list B [7] candidates list [8] path ball hand-overs
  // [9] routes list C [10] paths list C (the global-memory search tier)
  // [11] routes list B2 [12] paths list B2 (the group tier's hand-overs to the 512-slot wave tier)
  // [13] routes list B3 [14] paths list B3 (the 512-slot tier's hand-overs to the 4096-slot one)
  uint32_t* rl_routes_0;  // items the K2 ball tier hands to the search tiers (count ctl[1])
  uint32_t* ctl; uint32_t* rl_routes_a; uint32_t* rl_routes_b; uint32_t* rl_paths_a; uint32_t* rl_paths_b;
  uint32_t* rl_cand;
  uint32_t* rl_routes_c; uint32_t* rl_paths_c;
  uint32_t* trace_err;    // per trace: error bits of that trace only (the rest of the batch is unaffected)
  // locality order (round 4): state slots sorted by the Morton code of their point's coarse grid
  // cell; null = slot order.  K1 takes states, K2 items and the path stage pairs in this order
  // (a pair by its source state), so work that reads one region's cell records and route-ball
  // tables meets in one XCD's L2 instead of arriving in trace order from everywhere.
  const uint32_t* perm;
  const uint32_t* perm_paths;   // perm for the path stage too (null: the path stage takes slot order)
  uint32_t search_delta;        // cm: the wave tiers' delta-stepping width (kNone: plain rounds)
  // small runs (Matcher::run_small): the u64 totals the launches size themselves from on the
  // device (Workspace::tot64), the traversal-record capacity, and gate bits -- 1: K4, the report
  // and the segment gather skip a run whose path pool overflowed or whose records exceed seg_cap
  // (the host then runs the batch the ordinary way); 2: also one that handed searches to the
  // global-memory tier, which a small run does not launch before its scratch exists
  // 4: a steady run (Matcher::run_steady) sized from the pools an earlier run of the matcher left:
  // every stage after the transition scan skips a batch with more transitions or K2 sources than
  // trans_cap / src_cap (steady_abort), and the host re-runs it the ordinary way
  const unsigned long long* tot;
  uint64_t seg_cap;
  uint64_t trans_cap, src_cap;
  uint32_t gate;
};

__device__ __forceinline__ bool steady_abort(const DevBatch& b) {
  return (b.gate & 4u) && (b.tot[0] > b.trans_cap || b.tot[1] > b.src_cap);
}

__device__ __forceinline__ bool small_abort(const DevBatch& b) {
  if (!b.gate) return false;
  const uint32_t* c = b.ctl;
  return (c[2] & kErrPathOverflow) != 0u || ((b.gate & 2u) && (c[9] | c[10]) != 0u) || b.tot[2] > b.seg_cap ||
         steady_abort(b);
}

// A failure that belongs to one trajectory (too many roads in a radius, a search beyond every
// tier's capacity, a path that cannot be rebuilt) marks that trace only, as the reference fails
// one request (py/reporter_service.py:244-245) or skips one window (py/simple_reporter.py:169-173).
__device__ __forceinline__ void trace_fail(const DevBatch& b, uint64_t p, uint32_t bit) {
  atomicOr(&b.trace_err[b.slot_trace[p]], bit);
  atomicOr(&b.ctl[2], bit);
}

__device__ __forceinline__ bool edge_ok(uint32_t info, uint32_t acc) { return (((info >> 16) & 7u) & acc) != 0u; }
__device__ __forceinline__ uint64_t edge_key(const uint4& r, int mode) {
  return make_key(r.y, time_ms(r.y, mode_speed_dkph(mode, r.z & 0xffffu)));
}
__device__ __forceinline__ float as_f(uint32_t u) { return __uint_as_float(u); }

__device__ __forceinline__ float point_radius(const MatchOptions& o, float acc) {
  float r = o.search_radius;
  if (acc >= 0.0f && acc > r) r = acc;
  if (r > kMaxSearchRadius) r = kMaxSearchRadius;
  if (!(r > 0.0f)) r = 0.0f;
  return r;
}

// XCD-aware block order: the dispatcher deals workgroups round-robin over the 8 XCDs
// (block i runs on XCD i % 8), so consecutive work (the pairs of one trace) would land
// in 8 different L2s.  Renumber so each XCD gets one contiguous range of logical blocks.
__device__ __forceinline__ uint32_t xcd_block(uint32_t i, uint32_t n) {
  const uint32_t x = i & 7u, idx = i >> 3, q = n >> 3, r = n & 7u;
  return x < r ? x * (q + 1u) + idx : r * (q + 1u) + (x - r) * q + idx;
}

// bound on route distance (cm) for a layer pair: min(factor * gc, breakage)
__device__ __forceinline__ uint32_t route_bound(double gc, const MatchOptions& o) {
  double maxd = gc * (double)o.max_route_distance_factor;
  if ((double)o.breakage_distance < maxd) maxd = (double)o.breakage_distance;
  double bcm = floor(maxd * 100.0);
  if (!(bcm >= 0.0)) bcm = 0.0;
  return bcm > (double)kMaxBoundCm ? kMaxBoundCm : (uint32_t)bcm;
}
// The distance term of a transition with turn costs (rule 3b), exactly as the oracle's Viterbi
// forms it: turn weight U x factor x 2^-16 metres, plus |route_m - gc|; +inf for an invalid route.
// pair_info.w holds the pair's factor (float bits, 0: no turn costs).
__device__ __forceinline__ double route_term(uint32_t route_cm, uint32_t U, uint32_t factor_bits, double gc) {
  if (route_cm == kRouteInvalid) return __longlong_as_double(0x7ff0000000000000ll);
  const double tm = (double)U * ((double)__uint_as_float(factor_bits) * 0x1p-16);
  return tm + fabs((double)route_cm * 0.01 - gc);
}
__device__ __forceinline__ uint32_t time_bound(double dt, const MatchOptions& o) {
  if (!(dt > 0.0)) return 0xffffffffu;
  const double tm = floor(dt * (double)o.max_route_time_factor * 1000.0);
  return tm >= 4294967295.0 ? 0xffffffffu : (uint32_t)tm;
}

// ------------------------------------------------------------------------------------------
// Locality order (round 4).  On graphs whose route-ball tables and cell
// records are far larger than the L2s (C3: 4.2 GB of tables, C4: 68 GB), a step that visits
// states in trace order probes every table from vehicles spread over the whole step and all 8
// XCDs: each 16-byte row costs a 128-byte line from HBM (C3 K2 traffic 2.05x its algorithmic
// bytes, L2 hit rate 0.20).  The state slots are sorted once per step by the Morton code of
// their point's coarse grid cell; K1 reads its states, K2 its (pair, source) items and the path
// stage its chosen transitions in that order (a pair by its source state, whose exits own the
// tables it probes), with XCD-contiguous block ranges, and results still go to their slots.
// Results are identical in any order; only which L2 serves the reads changes.
__device__ __forceinline__ uint32_t morton_spread16(uint32_t v) {
  v &= 0xffffu;
  v = (v | (v << 8)) & 0x00ff00ffu;
  v = (v | (v << 4)) & 0x0f0f0f0fu;
  v = (v | (v << 2)) & 0x33333333u;
  v = (v | (v << 1)) & 0x55555555u;
  return v;
}
// The sort is a counting sort into kLocBuckets region buckets (a Morton-ordered 64 x 64 grid
// over the graph; one more bucket, last, for the slots without a state): three short passes
// (block histograms, one scan, block scatter) instead of a radix sort (hipcub's took 0.18 ms
// on C3 and 0.52 ms on C4 per 125 k traces).  Order inside a bucket is unspecified.
constexpr uint32_t kLocBucketBits = 12, kLocBuckets = 1u << kLocBucketBits;
constexpr uint32_t kLocPerThread = 16;   // slots per thread: a block of 256 threads covers 4096 slots
__device__ __forceinline__ uint32_t loc_bucket(const DevGraph& g, const DevBatch& b, uint64_t p, uint32_t shift) {
  const uint32_t k = b.slot_trace[p];
  const uint32_t o = b.trace_off[k];
  if ((uint32_t)(p - o) >= b.n_states[k]) return kLocBuckets;   // no state at this slot: last
  const uint32_t pt = o + b.state_orig[p];
  const double fx = floor(((double)b.lon[pt] - g.lon0) / g.dlon), fy = floor(((double)b.lat[pt] - g.lat0) / g.dlat);
  const uint32_t cx = fx < 0.0 ? 0u : (fx > (double)(g.ncx - 1) ? g.ncx - 1 : (uint32_t)fx);
  const uint32_t cy = fy < 0.0 ? 0u : (fy > (double)(g.ncy - 1) ? g.ncy - 1 : (uint32_t)fy);
  return morton_spread16(min(cx >> shift, 63u)) | (morton_spread16(min(cy >> shift, 63u)) << 1);
}
__global__ void __launch_bounds__(256) k_loc_count(DevGraph g, DevBatch b, uint32_t shift, uint16_t* key,
                                                   uint32_t* hist) {
  __shared__ uint32_t h[kLocBuckets + 1];
  for (uint32_t q = threadIdx.x; q <= kLocBuckets; q += 256) h[q] = 0u;
  __syncthreads();
  const uint64_t p0 = (uint64_t)blockIdx.x * (256u * kLocPerThread) + threadIdx.x;
#pragma unroll 4
  for (uint32_t i = 0; i < kLocPerThread; ++i) {
    const uint64_t p = p0 + 256u * i;
    if (p < b.P) {
      const uint32_t kk = loc_bucket(g, b, p, shift);
      key[p] = (uint16_t)kk;
      atomicAdd(&h[kk], 1u);
    }
  }
  __syncthreads();
  for (uint32_t q = threadIdx.x; q <= kLocBuckets; q += 256)
    if (h[q]) atomicAdd(&hist[q], h[q]);
}
// exclusive scan of the kLocBuckets + 1 bucket counts, in place (one block)
__global__ void __launch_bounds__(1024) k_loc_scan(uint32_t* hist) {
  __shared__ uint32_t ws[16];
  constexpr uint32_t per = (kLocBuckets + 1 + 1023) / 1024;
  const uint32_t q0 = threadIdx.x * per;
  uint32_t v[per], t = 0;
#pragma unroll
  for (uint32_t i = 0; i < per; ++i) { v[i] = q0 + i <= kLocBuckets ? hist[q0 + i] : 0u; t += v[i]; }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t incl = t;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(incl, d, 64);
    if (lane >= d) incl += u;
  }
  if (lane == 63) ws[wv] = incl;
  __syncthreads();
  uint32_t base = 0;
  for (int w = 0; w < wv; ++w) base += ws[w];
  uint32_t at = base + incl - t;
#pragma unroll
  for (uint32_t i = 0; i < per; ++i) {
    if (q0 + i <= kLocBuckets) hist[q0 + i] = at;
    at += v[i];
  }
}
__global__ void __launch_bounds__(256) k_loc_scatter(uint64_t P, const uint16_t* key, uint32_t* cursor, uint32_t* perm) {
  __shared__ uint32_t h[kLocBuckets + 1];
  for (uint32_t q = threadIdx.x; q <= kLocBuckets; q += 256) h[q] = 0u;
  __syncthreads();
  const uint64_t p0 = (uint64_t)blockIdx.x * (256u * kLocPerThread) + threadIdx.x;
  uint32_t kk[kLocPerThread], rk[kLocPerThread];
#pragma unroll
  for (uint32_t i = 0; i < kLocPerThread; ++i) {
    const uint64_t p = p0 + 256u * i;
    kk[i] = p < P ? key[p] : 0xffffu;
    rk[i] = kk[i] != 0xffffu ? atomicAdd(&h[kk[i]], 1u) : 0u;
  }
  __syncthreads();
  for (uint32_t q = threadIdx.x; q <= kLocBuckets; q += 256)
    if (h[q]) h[q] = atomicAdd(&cursor[q], h[q]);   // this block's range of the bucket
  __syncthreads();
#pragma unroll
  for (uint32_t i = 0; i < kLocPerThread; ++i)
    if (kk[i] != 0xffffu) perm[h[kk[i]] + rk[i]] = (uint32_t)(p0 + 256u * i);
}
// K2 items in locality order: item counts of the pairs whose source is perm[r] (their block
// partials for the scan; k_scan_apply_perm scatters the offsets to the pairs' src_off).  (Putting
// the counts at their ranks from k_trans_count instead, with per-256-rank atomics, measured 2-3x
// slower: the ranks of one region's slots are adjacent, so the atomics pile onto few addresses.)
__global__ void __launch_bounds__(256) k_perm_src_count(DevBatch b, uint32_t* pcnt, unsigned long long* part);
__global__ void __launch_bounds__(256) k_scan_apply_perm(const uint32_t* a, uint64_t n, const unsigned long long* part,
                                                         const uint32_t* perm, uint32_t* src_off);

// ------------------------------------------------------------------------------------------
// k_states: interpolation rule (points closer than interpolation_distance to the last
// state are not states; meili MapMatcher::OfflineMatch).  One wave per trace, 64 points per
// step: every lane computes, speculatively and in parallel, the distance from the point
// before it (d1) and from two points back (d2) — the two the sequential rule needs unless two
// points in a row are skipped.  The rule itself then walks the chunk with mask arithmetic:
// runs of d1 >= interp extend a run of states in one step, after a skipped point d2 decides,
// and only a second skip in a row computes a distance from the last state (wave-uniform).
__device__ __forceinline__ float lane_f(float v, uint32_t q) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)q));
}
__device__ __forceinline__ double lane_d(double v, uint32_t q) {
  const unsigned long long u = __double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, (int)q);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), (int)q);
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

__global__ void __launch_bounds__(64) k_states(DevBatch b) {
  const uint32_t k = blockIdx.x;
  if (k >= b.T) return;
  const int lane = threadIdx.x;
  // the run's control words and this trace's error bits start at zero (the first kernel of a run)
  if (lane == 0) b.trace_err[k] = 0u;
  if (k == 0 && lane < kCtlWords) b.ctl[lane] = 0u;
  const uint32_t o = b.trace_off[k], n = b.trace_off[k + 1] - o;
  const MatchOptions op = b.opts[b.trace_opt[k]];
  const double interp = (double)op.interpolation_distance;
  uint32_t ns = 0, last = 0;              // states so far, index of the last state
  float llon = 0.f, llat = 0.f;           // coordinates of the last state
  double lsin = 0.0, lcos = 0.0;          // and the sin / cos of its latitude (lat_sin / lat_cos)
  float c1lo = 0.f, c1la = 0.f, c2lo = 0.f, c2la = 0.f;   // points c0-1, c0-2
  // each chunk's coordinates load one chunk ahead, unconditionally at a clamped index (a
  // conditional load would be waited on where it is merged: a long trace's chunks then each
  // paid a memory round trip before their first instruction)
  const uint32_t nl = n ? n - 1u : 0u;
  float nlo = b.lon[o + min((uint32_t)lane, nl)], nla = b.lat[o + min((uint32_t)lane, nl)];
  // a chunk's stores are issued at the top of the next chunk, before its prefetch: vmcnt counts
  // loads and stores in issue order, so stores issued after a prefetch would make the next
  // chunk's wait for that prefetch wait for them too
  bool w_slot = false, w_state = false, w_gc = false;
  uint32_t w_i = 0, w_si = 0;
  double w_gcv = 0.0;
  for (uint32_t c0 = 0; c0 < n; c0 += 64) {
    const uint32_t i = c0 + lane, m = min(64u, n - c0);
    const bool act = i < n;
    float lo = act ? nlo : 0.f, la = act ? nla : 0.f;
    // the previous prefetch is consumed here, before the stores below are issued (its wait then
    // waits for nothing newer) and before the next prefetch (whose loads can then land in the
    // same registers instead of being copied at the back edge, a copy that waits for them)
    __asm__ volatile("" : "+v"(lo), "+v"(la) : : "memory");
    if (w_slot) b.slot_trace[o + w_i] = k;
    if (w_state) b.state_orig[o + w_si] = w_i;
    if (w_gc) b.gc[o + w_si] = w_gcv;
    __asm__ volatile("" : : : "memory");
    nlo = b.lon[o + min(i + 64u, nl)];
    nla = b.lat[o + min(i + 64u, nl)];
    w_slot = act;
    w_i = i;
    float lo1 = __shfl_up(lo, 1, 64), la1 = __shfl_up(la, 1, 64);
    float lo2 = __shfl_up(lo, 2, 64), la2 = __shfl_up(la, 2, 64);
    if (lane == 0) { lo1 = c1lo; la1 = c1la; lo2 = c2lo; la2 = c2la; }
    if (lane == 1) { lo2 = c1lo; la2 = c1la; }
    // sin / cos of each latitude once per lane, neighbours' by shuffle (the carried points
    // recompute theirs)
    const double s0 = lat_sin(la), k0 = lat_cos(la);
    double s1 = __shfl_up(s0, 1, 64), k1 = __shfl_up(k0, 1, 64), s2 = __shfl_up(s0, 2, 64), k2 = __shfl_up(k0, 2, 64);
    if (lane <= 1) {
      const float cl = lane == 0 ? c2la : c1la;
      s2 = lat_sin(cl); k2 = lat_cos(cl);
      if (lane == 0) { s1 = lat_sin(c1la); k1 = lat_cos(c1la); }
    }
    const double d1 = gc_trig(lo1, la1, s1, k1, lo, la, s0, k0);
    const double d2 = gc_trig(lo2, la2, s2, k2, lo, la, s0, k0);
    const bool a1 = act && (i == 0 || !(d1 < interp));
    const bool a2 = act && i >= 2 && !(d2 < interp);
    const unsigned long long A = __ballot(a1), B = __ballot(a2);
    unsigned long long st = 0;
    const uint32_t last0 = last;   // last state before this chunk
    double dx = 0.0;               // distance from the last state when two or more were skipped
    for (uint32_t q = 0; q < m;) {
      const uint32_t ii = c0 + q;
      if (ii == 0 || last + 1 == ii) {
        // a state right before: d1 decides; a run of d1 passes is a run of states
        const unsigned long long rest = ~(A >> q);
        const uint32_t run = min(rest ? (uint32_t)__builtin_ctzll(rest) : 64u, m - q);
        if (run) {
          st |= (run == 64u ? ~0ull : ((1ull << run) - 1ull)) << q;
          q += run;
          last = c0 + q - 1;
        } else {
          ++q;   // skipped: the next point is measured from two back
        }
        continue;
      }
      if (last + 2 == ii) {
        if ((B >> q) & 1ull) { st |= 1ull << q; last = ii; }
        ++q;
        continue;
      }
      // two or more skipped in a row: every remaining point of the chunk is measured from the
      // last state at once (one vector distance, the same function the one-point test used);
      // the first that is far enough is the next state, the ones before it are skipped
      float plo = llon, pla = llat;
      double ps = lsin, pc = lcos;
      if (last >= c0) {
        plo = lane_f(lo, last - c0); pla = lane_f(la, last - c0);
        ps = lane_d(s0, last - c0); pc = lane_d(k0, last - c0);
      }
      // gc_distance(plo, pla, lo, la) with both latitudes' sin / cos already at hand (the same
      // functions of the same floats: the same bits)
      const double dv = gc_trig(plo, pla, ps, pc, lo, la, s0, k0);
      const unsigned long long far = __ballot(act && !(dv < interp)) & (~0ull << q);
      if (!far) { q = m; break; }   // the rest of the chunk is skipped
      const uint32_t nq = (uint32_t)__builtin_ctzll(far);
      st |= 1ull << nq;
      last = c0 + nq;
      if (lane == (int)nq) dx = dv;
      q = nq + 1;
    }
    w_state = ((st >> lane) & 1ull) != 0ull;
    w_gc = false;
    if (w_state) {
      const unsigned long long below = st & ((1ull << lane) - 1ull);
      const uint32_t si = ns + (uint32_t)__popcll(below);
      w_si = si;   // state_orig[o + si] = i
      // gc from the previous state (the distance the rule just tested: d1, d2 or the explicit
      // one); k_trans_count and K3 read it instead of measuring it again
      if (si > 0) {
        const uint32_t prev = below ? c0 + 63u - (uint32_t)__builtin_clzll(below) : last0;
        w_gc = true;
        w_gcv = i - prev == 1u ? d1 : (i - prev == 2u ? d2 : dx);
      }
    }
    ns += (uint32_t)__popcll(st);
    if (last >= c0) {
      llon = lane_f(lo, last - c0); llat = lane_f(la, last - c0);
      lsin = lane_d(s0, last - c0); lcos = lane_d(k0, last - c0);
    }
    c1lo = lane_f(lo, 63); c1la = lane_f(la, 63);
    c2lo = lane_f(lo, 62); c2la = lane_f(la, 62);
  }
  if (w_slot) b.slot_trace[o + w_i] = k;
  if (w_state) b.state_orig[o + w_si] = w_i;
  if (w_gc) b.gc[o + w_si] = w_gcv;
  if (lane == 0) b.n_states[k] = ns;
}

// ------------------------------------------------------------------------------------------
// K1 k_candidates: one wave (64 lanes) per state slot.
struct CandSmem {
  uint32_t road[kCandH];
  unsigned long long best[kCandH];  // (sq bits << 32) | vertex  — lexicographic min per road
  uint32_t cell_lo[64], cell_hi[64];
  uint32_t used, ovf, ncell, slot_n;
  uint32_t list[kCandH];
};

// projection of the point onto the shape piece A->B in the point's local metric frame
// (A = {lon, lat, cum_cm}, B likewise); squared distance in m^2 and the offset along
// the road in cm.  Fixed operation order: bit-identical to oracle/meili_oracle.c.
__device__ __forceinline__ void project_rel(float ax, float ay, uint32_t acum, float bx, float by, uint32_t bcum,
                                            float& sq, uint32_t& s) {
  const float dx = bx - ax, dy = by - ay;
  const float l2 = dx * dx + dy * dy;
  float t = 0.0f;
  if (l2 > 0.0f) {
    t = -(ax * dx + ay * dy) / l2;
    if (t < 0.0f) t = 0.0f;
    if (t > 1.0f) t = 1.0f;
  }
  const float cx = ax + t * dx, cy = ay + t * dy;
  sq = cx * cx + cy * cy;
  const float along = (float)acum + t * (float)(bcum - acum);
  uint32_t v = (uint32_t)rintf(along);
  if (v < acum) v = acum;
  if (v > bcum) v = bcum;
  s = v;
}
__device__ __forceinline__ void project(float alon, float alat, uint32_t acum, float blon, float blat, uint32_t bcum,
                                        float lon, float lat, float mlon, float mlat, float& sq, uint32_t& s) {
  project_rel((alon - lon) * mlon, (alat - lat) * mlat, acum, (blon - lon) * mlon, (blat - lat) * mlat, bcum, sq, s);
}
// An item whose two endpoints lie beyond the padded radius on the same side in x or in y
//  cannot come within the radius: the projection lies between them, and the
// fp32 rounding of the projected point is far below pad - r >= 0.5 m (a few ulps of coordinates
// under 1000 km), so its sq exceeds r^2 with room to spare; rejecting it before the division is
// bit-exact.  Off by default: measured slower on C2 and CITY30 (the test diverges the lanes of
// a cell, and the division it saves is not what K1 waits on -- DESIGN.md §6 dead ends);
// -DRM_K1_REJECT=1 builds it.
#ifndef RM_K1_REJECT
#define RM_K1_REJECT 0
#endif
__device__ __forceinline__ bool outside_pad(float ax, float ay, float bx, float by, float pad) {
  if (!RM_K1_REJECT) return false;
  return (ax > pad && bx > pad) || (ax < -pad && bx < -pad) || (ay > pad && by > pad) || (ay < -pad && by < -pad);
}

// time_ms on the device: below 2^32 cm*360 the IEEE double quotient truncates to the exact
// floor (a non-integer quotient lies >= 1/dkph >= 2^-16 below the next integer, far above half
// an ulp, 2^-21); about half the instructions of the integer division
__device__ __forceinline__ uint32_t time_ms_dev(uint32_t d_cm, uint32_t dkph) {
  if (d_cm > 11930464u) return time_ms(d_cm, dkph);   // d_cm * 360 >= 2^32
  const uint32_t D = dkph ? dkph : 1u;
  return (uint32_t)((double)(d_cm * 360u) / (double)D);
}

// candidate descriptor of (road, s) for a travel mode: everything the route and path
// kernels need about a candidate in two dwordx4 (no dependent graph loads there)
__device__ __forceinline__ void desc_from_rec(const uint4& a, const uint4& c, uint32_t road, uint32_t s, int mode,
                                              uint32_t acc, uint4& d0, uint4& d1) {
  uint32_t spf = (a.w != kNone && edge_ok(c.y, acc)) ? mode_speed_dkph(mode, c.y & 0xffffu) : 0u;
  uint32_t spr = (c.x != kNone && edge_ok(c.z, acc)) ? mode_speed_dkph(mode, c.z & 0xffffu) : 0u;
  // a usable edge is never speed 0 here; time_ms() treats 0 as 1, so 1 keeps every result
  if (a.w != kNone && edge_ok(c.y, acc) && spf == 0u) spf = 1u;
  if (c.x != kNone && edge_ok(c.z, acc) && spr == 0u) spr = 1u;
  d0 = make_uint4(road, s, a.z, spf | (spr << 16));
  // d1 = {node0, node1, time_ms(s) entering forward from node0, time_ms(L - s) entering reverse from node1}
  d1 = make_uint4(a.x, a.y, spf ? time_ms_dev(s, spf) : 0xffffffffu, spr ? time_ms_dev(a.z - s, spr) : 0xffffffffu);
}

__device__ __forceinline__ void make_desc(const DevGraph& g, uint32_t road, uint32_t s, int mode, uint4& d0,
                                          uint4& d1) {
  desc_from_rec(g.road_rec[2 * (uint64_t)road], g.road_rec[2 * (uint64_t)road + 1], road, s, mode, mode_access(mode),
                d0, d1);
}

__device__ __forceinline__ void put_cand(const DevGraph& g, const DevBatch& b, uint64_t p, uint32_t rank, uint32_t road,
                                         uint32_t s, float sq, int mode) {
  uint4 d0, d1;
  make_desc(g, road, s, mode, d0, d1);
  const uint64_t at = p * kMaxCand + rank;
  b.cand_desc[2 * at] = d0;
  b.cand_desc[2 * at + 1] = d1;
  b.cand_sq[at] = sq;
}

// Unrolled loops over the per-lane slot arrays stop as soon as no active lane needs the
// slot (a scalar branch on a ballot) instead of always walking all kMaxCand slots.
#define K1_UNIFORM_STOP(c) (__ballot(c) == 0ull)

// K1 lane tier: one lane per state.  Cell items are read as cell-major 32-byte records
// (both shape vertices + road + access bits), so a test is two dwordx4 loads with no
// dependent lookup.  Per-road minima live in 16 registers; a state with more roads
// inside its radius is queued for the wave tier (k_candidates_wave).
#ifndef RM_K1_ROWS
#define RM_K1_ROWS 4
#endif
constexpr int kK1Rows = RM_K1_ROWS;   // grid rows whose items K1 walks as one sequence
#ifndef RM_K1_BATCH
#define RM_K1_BATCH 4
#endif
constexpr int kK1Batch = RM_K1_BATCH;  // cell records loaded together per lane
// per-road minima the lane tier keeps in registers; a state with more roads inside its radius goes
// to the wave tier (its LDS hash holds any number; the same candidates either way)
#ifndef RM_K1_SLOTS
#define RM_K1_SLOTS 16
#endif
constexpr int kK1Slots = RM_K1_SLOTS;
static_assert(kK1Slots % 4 == 0 && kK1Slots <= kMaxCand, "K1 slots");
#ifndef RM_K1_WPE
#define RM_K1_WPE 1
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RM_K1_WPE))) k_candidates_lane(DevGraph g, DevBatch b) {
  uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b.perm) {   // locality order: each XCD walks one contiguous range of the sorted states
    const uint64_t r = (uint64_t)xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    if (r >= b.P) return;
    p = b.perm[r];
  }
  if (p >= b.P) return;
  const uint32_t k = b.slot_trace[p];
  const uint32_t o = b.trace_off[k];
  const uint32_t s = (uint32_t)(p - o);
  if (s >= b.n_states[k]) return;
  const MatchOptions op = b.opts[b.trace_opt[k]];
  const uint32_t acc = mode_access(op.mode);
  const uint32_t pt = o + b.state_orig[p];
  const float lon = b.lon[pt], lat = b.lat[pt];
  const float r = point_radius(op, b.acc[pt]);
  const float mlon = meters_per_lon(lat);
  const float mlat = (float)kMetersPerDegLat;
  const float r2 = r * r;
  const float pad = r * 1.01f + 0.5f;
  const float qlon = pad / mlon, qlat = pad / mlat;
  const double fx0 = floor(((double)(lon - qlon) - g.lon0) / g.dlon);
  const double fx1 = floor(((double)(lon + qlon) - g.lon0) / g.dlon);
  const double fy0 = floor(((double)(lat - qlat) - g.lat0) / g.dlat);
  const double fy1 = floor(((double)(lat + qlat) - g.lat0) / g.dlat);
  uint32_t rroad[kK1Slots], rs[kK1Slots];
  unsigned long long rbest[kK1Slots];
  uint32_t n = 0;
  bool ovf = false;
  if (!(fx1 < 0 || fy1 < 0 || fx0 > (double)(g.ncx - 1) || fy0 > (double)(g.ncy - 1))) {
    const uint32_t x0 = fx0 < 0 ? 0u : (uint32_t)fx0, y0 = fy0 < 0 ? 0u : (uint32_t)fy0;
    const uint32_t x1 = fx1 > (double)(g.ncx - 1) ? g.ncx - 1 : (uint32_t)fx1;
    const uint32_t y1 = fy1 > (double)(g.ncy - 1) ? g.ncy - 1 : (uint32_t)fy1;
    // the items of cells x0..x1 of one grid row are one contiguous range (cell-major CSR).
    // Rows go kK1Rows at a time: the window's row ranges are read at once and its rows' items
    // are walked as ONE sequence, four records per batch across row boundaries (clamped,
    // branch-free loads, so the loads of a batch overlap instead of paying one round trip per
    // item or per row)
    for (uint32_t w0 = y0; w0 <= y1 && !ovf; w0 += kK1Rows) {
      const uint32_t nrow = min(y1 - w0 + 1u, (uint32_t)kK1Rows);
      uint32_t ra[kK1Rows], re[kK1Rows], base[kK1Rows], end[kK1Rows];
#pragma unroll
      for (int r = 0; r < kK1Rows; ++r) {
        const uint32_t cy = w0 + min((uint32_t)r, nrow - 1u);
        ra[r] = g.cell_off[cy * g.ncx + x0];
        re[r] = g.cell_off[cy * g.ncx + x1 + 1];
      }
      uint32_t tot = 0;
#pragma unroll
      for (int r = 0; r < kK1Rows; ++r) {
        base[r] = ra[r] - tot;   // item of sequence index q in row r: base[r] + q
        tot += (uint32_t)r < nrow ? re[r] - ra[r] : 0u;
        end[r] = tot;
      }
      for (uint32_t q0 = 0; q0 < tot && !ovf; q0 += kK1Batch) {
        uint4 r0[kK1Batch], r1[kK1Batch];
#pragma unroll
        for (int y = 0; y < kK1Batch; ++y) {
          const uint32_t q = min(q0 + (uint32_t)y, tot - 1u);
          uint32_t bq = base[0];
#pragma unroll
          for (int r = 1; r < kK1Rows; ++r)
            if (q >= end[r - 1]) bq = base[r];
          const uint64_t it = bq + q;
          r0[y] = g.cell_rec[2 * it];
          r1[y] = g.cell_rec[2 * it + 1];
        }
#pragma unroll
        for (int y = 0; y < kK1Batch; ++y) {
          if (q0 + y >= tot || ovf) break;
          if (!((r1[y].z >> 29) & acc)) continue;
          const float ax = (as_f(r0[y].x) - lon) * mlon, ay = (as_f(r0[y].y) - lat) * mlat;
          const float bx = (as_f(r0[y].z) - lon) * mlon, by = (as_f(r0[y].w) - lat) * mlat;
          if (outside_pad(ax, ay, bx, by, pad)) continue;
          float sq; uint32_t sc;
          project_rel(ax, ay, r1[y].x, bx, by, r1[y].y, sq, sc);
          if (!(sq <= r2)) continue;
          const uint32_t road = r1[y].z & 0x1fffffffu;
          const unsigned long long key = ((unsigned long long)__float_as_uint(sq) << 32) | r1[y].w;
          bool found = false;
#pragma unroll
          for (int x = 0; x < kK1Slots; ++x) {
            if (K1_UNIFORM_STOP(x < (int)n)) break;   // no active lane holds slot x yet
            if (x < (int)n && rroad[x] == road) {
              found = true;
              if (key < rbest[x]) { rbest[x] = key; rs[x] = sc; }
            }
          }
          if (found) continue;
          if (n >= (uint32_t)kK1Slots) { ovf = true; break; }
#pragma unroll
          for (int x = 0; x < kK1Slots; ++x) {
            if (K1_UNIFORM_STOP(x <= (int)n)) break;
            if (x == (int)n) { rroad[x] = road; rbest[x] = key; rs[x] = sc; }
          }
          ++n;
        }
      }
    }
  }
  if (ovf) {
    const uint32_t q = atomicAdd(&b.ctl[7], 1u);
    b.rl_cand[q] = (uint32_t)p;
    return;
  }
  // rank by (sq, road); descriptors are written four at a time after their road records
  // have all arrived (a store between two loads would serialise them: shared vmcnt)
  const uint32_t cacc = mode_access(op.mode);
#pragma unroll
  for (int x0 = 0; x0 < kK1Slots; x0 += 4) {
    if (K1_UNIFORM_STOP(x0 < (int)n)) break;
    if (x0 >= (int)n) break;
    uint4 ra[4], rc[4];
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      const uint64_t road = rroad[min(x0 + y, (int)n - 1)];
      ra[y] = g.road_rec[2 * road];
      rc[y] = g.road_rec[2 * road + 1];
    }
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      const int x = x0 + y;
      if (x >= (int)n) break;
      const uint32_t sqb = (uint32_t)(rbest[x] >> 32);
      // rank by (sq, road): both fit one u64 key (sq >= 0, so its bits order as the value)
      const unsigned long long kx = ((unsigned long long)sqb << 32) | rroad[x];
      uint32_t rank = 0;
#pragma unroll
      for (int z = 0; z < kK1Slots; ++z) {
        if (K1_UNIFORM_STOP(z < (int)n)) break;
        if (z >= (int)n) continue;
        rank += ((((rbest[z] >> 32) << 32) | rroad[z]) < kx) ? 1u : 0u;
      }
      uint4 d0, d1;
      desc_from_rec(ra[y], rc[y], rroad[x], rs[x], op.mode, cacc, d0, d1);
      const uint64_t at = p * kMaxCand + rank;
      b.cand_desc[2 * at] = d0;
      b.cand_desc[2 * at + 1] = d1;
      b.cand_sq[at] = __uint_as_float(sqb);
    }
  }
  b.cand_n[p] = (uint8_t)n;
}

// wave tier of K1: states whose radius holds more roads than the lane tier keeps
__device__ void cand_wave_one(const DevGraph& g, const DevBatch& b, CandSmem& sm, uint64_t p) {
  const int lane = threadIdx.x;
  const uint32_t k = b.slot_trace[p];
  const uint32_t o = b.trace_off[k];
  const MatchOptions op = b.opts[b.trace_opt[k]];
  const uint32_t acc = mode_access(op.mode);
  const uint32_t pt = o + b.state_orig[p];
  const float lon = b.lon[pt], lat = b.lat[pt];
  const float r = point_radius(op, b.acc[pt]);
  const float mlon = meters_per_lon(lat);
  const float mlat = (float)kMetersPerDegLat;
  const float r2 = r * r;
  const float pad = r * 1.01f + 0.5f;
  const float qlon = pad / mlon, qlat = pad / mlat;
  const double fx0 = floor(((double)(lon - qlon) - g.lon0) / g.dlon);
  const double fx1 = floor(((double)(lon + qlon) - g.lon0) / g.dlon);
  const double fy0 = floor(((double)(lat - qlat) - g.lat0) / g.dlat);
  const double fy1 = floor(((double)(lat + qlat) - g.lat0) / g.dlat);
  for (int h = lane; h < kCandH; h += kWave) { sm.road[h] = kEmpty; sm.best[h] = ~0ull; }
  if (lane == 0) { sm.used = 0; sm.ovf = 0; }
  __syncthreads();
  uint32_t n_found = 0;
  if (!(fx1 < 0 || fy1 < 0 || fx0 > (double)(g.ncx - 1) || fy0 > (double)(g.ncy - 1))) {
    const uint32_t x0 = fx0 < 0 ? 0u : (uint32_t)fx0, y0 = fy0 < 0 ? 0u : (uint32_t)fy0;
    const uint32_t x1 = fx1 > (double)(g.ncx - 1) ? g.ncx - 1 : (uint32_t)fx1;
    const uint32_t y1 = fy1 > (double)(g.ncy - 1) ? g.ncy - 1 : (uint32_t)fy1;
    const uint32_t nx = x1 - x0 + 1, ncell = nx * (y1 - y0 + 1);
    // the covered cells, 64 at a time: their item ranges and an inclusive scan of their item
    // counts go to LDS, and the cells' items are walked as ONE sequence, a lane per item (a
    // point's few cells cost one round of loads, not one per cell)
    for (uint32_t c0 = 0; c0 < ncell; c0 += kWave) {
      const uint32_t c = c0 + lane;
      uint32_t lo = 0, cnt = 0;
      if (c < ncell) {
        const uint32_t cell = (y0 + c / nx) * g.ncx + (x0 + c % nx);
        lo = g.cell_off[cell];
        cnt = g.cell_off[cell + 1] - lo;
      }
      uint32_t incl = cnt;
#pragma unroll
      for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t u = __shfl_up(incl, d, kWave);
        if (lane >= d) incl += u;
      }
      const uint32_t tot = (uint32_t)__shfl((int)incl, kWave - 1, kWave);
      sm.cell_lo[lane] = lo;
      sm.cell_hi[lane] = incl;   // here: the inclusive item prefix of the staged cells
      __syncthreads();
      {
        for (uint32_t f = lane; f < tot; f += kWave) {
          uint32_t a = 0, e = kWave - 1;   // the staged cell holding item f: first prefix > f
          while (a < e) {
            const uint32_t mid = (a + e) >> 1;
            if (sm.cell_hi[mid] > f) e = mid;
            else a = mid + 1;
          }
          const uint32_t it = sm.cell_lo[a] + (f - (a ? sm.cell_hi[a - 1] : 0u));
          const uint4 r0 = g.cell_rec[2 * (uint64_t)it], r1 = g.cell_rec[2 * (uint64_t)it + 1];
          if (!((r1.z >> 29) & acc)) continue;
          const float ax = (as_f(r0.x) - lon) * mlon, ay = (as_f(r0.y) - lat) * mlat;
          const float bx = (as_f(r0.z) - lon) * mlon, by = (as_f(r0.w) - lat) * mlat;
          if (outside_pad(ax, ay, bx, by, pad)) continue;
          float sq; uint32_t sc;
          project_rel(ax, ay, r1.x, bx, by, r1.y, sq, sc);
          if (!(sq <= r2)) continue;
          const uint32_t road = r1.z & 0x1fffffffu, v = r1.w;
          // per-road min (sq, vertex) in the LDS hash
          uint32_t h = (road * 2654435761u) & (kCandH - 1);
          for (int probe = 0; probe < kCandH; ++probe) {
            uint32_t cur = sm.road[h];
            if (cur == kEmpty) {
              cur = atomicCAS(&sm.road[h], kEmpty, road);
              if (cur == kEmpty) {
                const uint32_t u = atomicAdd(&sm.used, 1u);
                sm.list[u] = h;
                cur = road;
              }
            }
            if (cur == road) {
              atomicMin(&sm.best[h], ((unsigned long long)__float_as_uint(sq) << 32) | v);
              break;
            }
            h = (h + 1) & (kCandH - 1);
          }
        }
      }
      __syncthreads();
    }
    n_found = sm.used;
  }
  if (n_found > kCandH * 3 / 4) {  // too many roads inside the radius
    if (lane == 0) trace_fail(b, p, kErrCandOverflow);
    n_found = 0;
  }
  // rank by (sq, road); keep the first 16
  for (uint32_t q = lane; q < n_found; q += kWave) {
    const uint32_t h = sm.list[q];
    const uint32_t road = sm.road[h];
    const unsigned long long bst = sm.best[h];
    const uint32_t sqb = (uint32_t)(bst >> 32);
    uint32_t rank = 0;
    for (uint32_t q2 = 0; q2 < n_found; ++q2) {
      const uint32_t h2 = sm.list[q2];
      const uint32_t sqb2 = (uint32_t)(sm.best[h2] >> 32), road2 = sm.road[h2];
      rank += (sqb2 < sqb || (sqb2 == sqb && road2 < road)) ? 1u : 0u;
    }
    if (rank < (uint32_t)kMaxCand) {
      const uint32_t v = (uint32_t)bst;
      const uint4 A = g.verts[v], B = g.verts[v + 1];
      float sq; uint32_t sc;
      project(as_f(A.x), as_f(A.y), A.z, as_f(B.x), as_f(B.y), B.z, lon, lat, mlon, mlat, sq, sc);
      put_cand(g, b, p, rank, road, sc, sq, op.mode);
    }
  }
  if (lane == 0) b.cand_n[p] = (uint8_t)min(n_found, (uint32_t)kMaxCand);
}

// all = 0: the lane tier's hand-overs (ctl[7]); all = 1: every state slot of the batch (small
// runs: one wave per state is a few rounds of loads where a lane walks its cells one by one)
__global__ void __launch_bounds__(64) k_candidates_wave(DevGraph g, DevBatch b, int all) {
  __shared__ CandSmem sm;
  const uint32_t n_items = all ? (uint32_t)b.P : min(b.ctl[7], (uint32_t)b.P);
  for (uint32_t item = blockIdx.x; item < n_items; item += gridDim.x) {
    const uint32_t p = all ? item : b.rl_cand[item];
    if (all) {
      const uint32_t k = b.slot_trace[p];
      if (p - b.trace_off[k] >= b.n_states[k]) continue;   // not a state slot (block-uniform)
    }
    cand_wave_one(g, b, sm, p);
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// u64 sums of two per-lane values: the u32 exclusive scans that lay out routes and records
// would wrap silently past 2^32, so the host checks these totals instead of off + cnt.
// Each 256-thread block writes its pair of partials to part[2 * block]; k_scan_parts turns
// them into block offsets and totals.  (One same-address u64 atomic per block serialises at
// ~12 ns across the 8 XCDs: 23 k blocks of C2 cost 0.57 ms that way.)
__device__ __forceinline__ void block_sum2_u64(unsigned long long a, unsigned long long c, unsigned long long* part) {
  __shared__ unsigned long long sa[4], sc[4];
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    a += __shfl_down(a, d, 64);
    c += __shfl_down(c, d, 64);
  }
  if ((threadIdx.x & 63) == 0) { sa[threadIdx.x >> 6] = a; sc[threadIdx.x >> 6] = c; }
  __syncthreads();
  if (threadIdx.x == 0)
    reinterpret_cast<ulonglong2*>(part)[blockIdx.x] =
        make_ulonglong2(sa[0] + sa[1] + sa[2] + sa[3], sc[0] + sc[1] + sc[2] + sc[3]);
}

// Exclusive scans of per-slot counts from the block partials the counting kernels already
// produce (k_trans_count: pairs per 256 slots, k_sum_u64: per 1024): k_scan_parts turns the
// partial pairs into block offsets in place (one block) and writes the u64 totals; the apply
// kernels scan each block locally and add its offset.  Three short passes instead of a
// generic device scan per array.
__device__ __forceinline__ void block_excl_scan2(unsigned long long a, unsigned long long c, unsigned long long& ea,
                                                 unsigned long long& ec, unsigned long long* sa, unsigned long long* sc,
                                                 int nwaves) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned long long ia = a, ic = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long ta = __shfl_up(ia, d, 64), tc = __shfl_up(ic, d, 64);
    if (lane >= d) { ia += ta; ic += tc; }
  }
  if (lane == 63) { sa[wv] = ia; sc[wv] = ic; }
  __syncthreads();
  unsigned long long ba = 0, bc = 0;
  for (int w = 0; w < nwaves; ++w) {
    const unsigned long long xa = sa[w], xc = sc[w];
    ba += w < wv ? xa : 0ull;
    bc += w < wv ? xc : 0ull;
  }
  ea = ba + ia - a;
  ec = bc + ic - c;
}

__global__ void __launch_bounds__(1024) k_scan_parts(unsigned long long* part, uint32_t nb, unsigned long long* out) {
  __shared__ unsigned long long sa[16], sc[16];
  const uint32_t per = (nb + 1023u) / 1024u;
  const uint32_t b0 = min(threadIdx.x * per, nb), b1 = min(b0 + per, nb);
  ulonglong2* pp = reinterpret_cast<ulonglong2*>(part);
  unsigned long long a = 0, c = 0;
#pragma unroll 8
  for (uint32_t q = b0; q < b1; ++q) { const ulonglong2 v = pp[q]; a += v.x; c += v.y; }
  unsigned long long ea, ec;
  block_excl_scan2(a, c, ea, ec, sa, sc, 16);
#pragma unroll 8
  for (uint32_t q = b0; q < b1; ++q) {
    const ulonglong2 v = pp[q];
    pp[q] = make_ulonglong2(ea, ec);
    ea += v.x;
    ec += v.y;
  }
  if (threadIdx.x == 1023) { out[0] = ea; out[1] = ec; }
}

// one count of each array per thread, blocks of 256 (k_trans_count's partials); a block's
// counts sum to < 2^32 (at most 256 x 16 x 16), so the in-block scan runs on u32 pairs
__global__ void __launch_bounds__(256) k_scan_apply2(const uint32_t* a, const uint32_t* c, uint64_t n,
                                                     const unsigned long long* part, uint32_t* ao, uint32_t* co) {
  __shared__ uint32_t sa[4], sc[4];
  const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const ulonglong2 base = reinterpret_cast<const ulonglong2*>(part)[blockIdx.x];
  const uint32_t va = p < n ? a[p] : 0u, vc = p < n ? c[p] : 0u;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t ia = va, ic = vc;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t ta = __shfl_up(ia, d, 64), tc = __shfl_up(ic, d, 64);
    if (lane >= d) { ia += ta; ic += tc; }
  }
  if (lane == 63) { sa[wv] = ia; sc[wv] = ic; }
  __syncthreads();
  uint32_t ba = 0, bc = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    ba += w < wv ? sa[w] : 0u;
    bc += w < wv ? sc[w] : 0u;
  }
  if (p < n) {
    ao[p] = (uint32_t)base.x + ba + ia - va;
    co[p] = (uint32_t)base.y + bc + ic - vc;
  }
}

// four counts per thread, blocks of 256 (k_sum_u64's partials)
__global__ void __launch_bounds__(256) k_scan_apply4(const uint32_t* a, uint64_t n, const unsigned long long* part,
                                                     uint32_t* ao) {
  __shared__ unsigned long long sa[4], sc[4];
  const uint64_t i = ((uint64_t)blockIdx.x * 256u + threadIdx.x) * 4u;
  uint32_t v[4] = {0u, 0u, 0u, 0u};
  if (i + 4 <= n) {
    const uint4 q = *reinterpret_cast<const uint4*>(a + i);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
    for (uint64_t x = i; x < n; ++x) v[x - i] = a[x];
  }
  unsigned long long ea, ec;
  block_excl_scan2((unsigned long long)v[0] + v[1] + v[2] + v[3], 0ull, ea, ec, sa, sc, 4);
  const unsigned long long base = part[2 * blockIdx.x] + ea;
  const uint32_t o0 = (uint32_t)base, o1 = o0 + v[0], o2 = o1 + v[1], o3 = o2 + v[2];
  if (i + 4 <= n) {
    *reinterpret_cast<uint4*>(ao + i) = make_uint4(o0, o1, o2, o3);
  } else {
    const uint32_t o[4] = {o0, o1, o2, o3};
    for (uint64_t x = i; x < n; ++x) ao[x] = o[x - i];
  }
}

__global__ void __launch_bounds__(256) k_perm_src_count(DevBatch b, uint32_t* pcnt, unsigned long long* part) {
  const uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  uint32_t c = 0;
  if (r < b.P) {   // every lane reaches the block sum (it holds a barrier)
    const uint64_t q = (uint64_t)b.perm[r] + 1u;   // the pair whose source state is perm[r]
    c = q < b.P ? b.src_cnt[q] : 0u;               // 0 unless q is a pair of the same trace
    pcnt[r] = c;
  }
  block_sum2_u64(c, 0ull, part);
}
__global__ void __launch_bounds__(256) k_scan_apply_perm(const uint32_t* a, uint64_t n, const unsigned long long* part,
                                                         const uint32_t* perm, uint32_t* src_off) {
  __shared__ uint32_t sa[4];
  const uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const uint32_t base = (uint32_t)reinterpret_cast<const ulonglong2*>(part)[blockIdx.x].x;
  const uint32_t v = r < n ? a[r] : 0u;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t iv = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(iv, d, 64);
    if (lane >= d) iv += t;
  }
  if (lane == 63) sa[wv] = iv;
  __syncthreads();
  uint32_t bb = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) bb += w < wv ? sa[w] : 0u;
  if (r < n && v) src_off[perm[r] + 1u] = base + bb + iv - v;
}

// transition counts for the exclusive scan that lays out route[] compactly, plus the
// per-pair constants K2 needs (bounds, candidate counts, mode) in one dwordx4; the block
// partials of the u64 totals of transitions and (pair, source) items go to part[]
__global__ void __launch_bounds__(256) k_trans_count(DevBatch b, unsigned long long* part) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t c = 0, ns = 0;
  if (p < b.P) {   // every lane reaches the block sum below (it holds a barrier)
    b.choice[p] = -1;      // K3 sets the chosen candidates; the path stage counts chosen transitions
    b.path_cnt[p] = 0u;
    const uint32_t k = b.slot_trace[p];
    const uint32_t o = b.trace_off[k];
    const uint32_t s = (uint32_t)(p - o);
    const uint32_t S = b.n_states[k];
    if (s < S) b.state_time[p] = b.time[o + b.state_orig[p]];   // K4 reads the state times by slot
    if (s >= 1 && s < S) {
      const uint32_t KA = b.cand_n[p - 1], KB = b.cand_n[p];
      c = KA * KB;
      ns = KB ? KA : 0u;
      const uint32_t pa = o + b.state_orig[p - 1], pb = o + b.state_orig[p];
      const double gc = b.gc[p];   // written by k_states (the rule's own measurement)
      const MatchOptions op = b.opts[b.trace_opt[k]];
      // .w: the pair's turn_penalty_factor (float bits) when its routes carry turn costs (rule 3b), else 0
      b.pair_info[p] = make_uint4(route_bound(gc, op), time_bound(b.time[pb] - b.time[pa], op),
                                  KA | (KB << 8) | ((uint32_t)op.mode << 16),
                                  op.turn_penalty_factor > 0.f ? __float_as_uint(op.turn_penalty_factor) : 0u);
    }
    b.trans_cnt[p] = c;
    b.src_cnt[p] = ns;
  }
  block_sum2_u64(c, ns, part);
}

// one work item per (layer pair, source candidate): item -> pair slot
__global__ void k_src_items(DevBatch b) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= b.P) return;
  const uint32_t n = b.src_cnt[p], at = b.src_off[p];
  for (uint32_t i = 0; i < n; ++i) b.src_item[at + i] = (uint32_t)p;
}

// ---- small runs (Matcher::run_small): one kernel in place of k_scan_parts + an apply pass (+
// k_src_items / k_rec_slot).  A small batch has at most a few hundred partials, so each block
// folds the partials before its own (and block 0 all of them, for the totals) instead of
// waiting for a separate one-block scan: three launches fewer per stage, ~5 us each.
__device__ __forceinline__ void block_prefix_parts(const unsigned long long* part, uint32_t nb, uint32_t upto,
                                                   unsigned long long* pre, unsigned long long* all) {
  __shared__ unsigned long long s[4][4];
  unsigned long long a = 0, c = 0, ta = 0, tc = 0;
  const ulonglong2* pp = reinterpret_cast<const ulonglong2*>(part);
  for (uint32_t q = threadIdx.x; q < nb; q += blockDim.x) {
    const ulonglong2 v = pp[q];
    ta += v.x; tc += v.y;
    if (q < upto) { a += v.x; c += v.y; }
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    a += __shfl_down(a, d, 64); c += __shfl_down(c, d, 64);
    ta += __shfl_down(ta, d, 64); tc += __shfl_down(tc, d, 64);
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { s[wv][0] = a; s[wv][1] = c; s[wv][2] = ta; s[wv][3] = tc; }
  __syncthreads();
  for (int j = 0; j < 4; ++j) {
    unsigned long long x = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) x += s[w][j];
    if (j < 2) pre[j] = x; else all[j - 2] = x;
  }
}

// k_scan_apply2 + k_src_items over k_trans_count's partials (blocks of 256 pairs); totals to tot[0..1]
__global__ void __launch_bounds__(256) k_trans_apply_small(DevBatch b, const unsigned long long* part, uint32_t nb,
                                                           unsigned long long* tot) {
  unsigned long long pre[2], all[2];
  block_prefix_parts(part, nb, blockIdx.x, pre, all);
  if (blockIdx.x == 0 && threadIdx.x == 0) { tot[0] = all[0]; tot[1] = all[1]; }
  __shared__ uint32_t sa[4], sc[4];
  const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const uint32_t va = p < b.P ? b.trans_cnt[p] : 0u, vc = p < b.P ? b.src_cnt[p] : 0u;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t ia = va, ic = vc;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t ta = __shfl_up(ia, d, 64), tc = __shfl_up(ic, d, 64);
    if (lane >= d) { ia += ta; ic += tc; }
  }
  if (lane == 63) { sa[wv] = ia; sc[wv] = ic; }
  __syncthreads();
  uint32_t ba = 0, bc = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    ba += w < wv ? sa[w] : 0u;
    bc += w < wv ? sc[w] : 0u;
  }
  if (p < b.P) {
    const uint32_t at = (uint32_t)pre[1] + bc + ic - vc;
    b.trans_off[p] = (uint32_t)pre[0] + ba + ia - va;
    b.src_off[p] = at;
    for (uint32_t i = 0; i < vc; ++i) b.src_item[at + i] = (uint32_t)p;
  }
}

// k_scan_apply4 + k_rec_slot over k_sum_u64's partials (blocks of 1024 slots); total to tot[2].
// Records past seg_cap are not written (the run is then gated off: small_abort).
__global__ void __launch_bounds__(256) k_path_apply_small(DevBatch b, const unsigned long long* part, uint32_t nb,
                                                          unsigned long long* tot, uint32_t* rec_slot) {
  unsigned long long pre[2], all[2];
  block_prefix_parts(part, nb, blockIdx.x, pre, all);
  if (blockIdx.x == 0 && threadIdx.x == 0) tot[2] = all[0];
  __shared__ unsigned long long sa[4], sc[4];
  const uint64_t n = b.P;
  const uint64_t i = ((uint64_t)blockIdx.x * 256u + threadIdx.x) * 4u;
  uint32_t v[4] = {0u, 0u, 0u, 0u};
  for (uint64_t x = i; x < n && x < i + 4; ++x) v[x - i] = b.path_cnt[x];
  unsigned long long ea, ec;
  block_excl_scan2((unsigned long long)v[0] + v[1] + v[2] + v[3], 0ull, ea, ec, sa, sc, 4);
  uint64_t o = pre[0] + ea;
  for (uint64_t x = i; x < n && x < i + 4; ++x) {
    b.trav_off[x] = (uint32_t)o;
    const uint32_t c = v[x - i];
    for (uint32_t q = 0; q < c; ++q)
      if (o + q < b.seg_cap) rec_slot[o + q] = (uint32_t)x;
    o += c;
  }
}

// Compaction for the downloads: trace k's records [base[k], base[k] + cnt[k]) of a per-trace
// pool (sized by traversal records, mostly empty) to dst[off[k] ..), one wave per trace, u64
// words.  The boundary then moves only the records (C2: 15 MB of segments, not a 362 MB pool).
__global__ void __launch_bounds__(64) k_gather_recs(uint32_t T, const uint32_t* base, const uint32_t* cnt,
                                                    const uint32_t* off, const unsigned long long* src, uint32_t words,
                                                    unsigned long long* dst) {
  for (uint32_t k = blockIdx.x; k < T; k += gridDim.x) {
    const uint64_t n = (uint64_t)cnt[k] * words;
    const unsigned long long* s = src + (uint64_t)base[k] * words;
    unsigned long long* d = dst + (uint64_t)off[k] * words;
    for (uint64_t q = threadIdx.x; q < n; q += 64) d[q] = s[q];
  }
}

// the per-trace segment offsets of a small run's reply (exclusive scan of seg_cnt, T + 1 words;
// one block) -- all zero, and seg_cnt zeroed, when the run is gated off
__global__ void __launch_bounds__(1024) k_seg_offsets_small(DevBatch b, uint32_t* off) {
  __shared__ unsigned long long sa[16], sc[16];
  const uint32_t T = b.T;
  const bool off_gate = small_abort(b);
  const uint32_t per = (T + 1023u) / 1024u;
  const uint32_t k0 = min(threadIdx.x * per, T), k1 = min(k0 + per, T);
  unsigned long long a = 0;
  for (uint32_t k = k0; k < k1; ++k) a += off_gate ? 0u : b.seg_cnt[k];
  unsigned long long ea, ec;
  block_excl_scan2(a, 0ull, ea, ec, sa, sc, 16);
  for (uint32_t k = k0; k < k1; ++k) {
    off[k] = (uint32_t)ea;
    if (off_gate) b.seg_cnt[k] = 0u;
    else ea += b.seg_cnt[k];
  }
  if (threadIdx.x == 1023) off[T] = (uint32_t)ea;
}

// descriptor field access (see Workspace::cand_desc)
__device__ __forceinline__ uint32_t d_spf(const uint4& d0) { return d0.w & 0xffffu; }
__device__ __forceinline__ uint32_t d_spr(const uint4& d0) { return d0.w >> 16; }

// route key from a source candidate a to a target candidate b given a label lookup
// (dist, time of the shortest route to a node); combos in the oracle's fixed order:
// direct forward, direct reverse, entry forward (via node0), entry reverse (via node1)
// (lab0, lab1 = labels of the target road's node0 / node1; read only when the direction is usable)
__device__ __forceinline__ unsigned long long route_key_vals(const uint4& a0, const uint4& b0, const uint4& b1,
                                                             unsigned long long lab0, unsigned long long lab1,
                                                             int* combo) {
  const uint32_t sa = a0.y, rb = b0.x, sb = b0.y, L = b0.z, spf = d_spf(b0), spr = d_spr(b0);
  unsigned long long best = kKeyInf;
  int bc = -1;
  if (a0.x == rb) {
    // direct along the road: forward when s_b > s_a, reverse when s_b < s_a; at s_b == s_a both
    // give (0, 0) and forward comes first -- so one division decides it (a second, divergent
    // fp64 division per transition cost K2 9 % on C2)
    const bool fw = sb > sa || (sb == sa && spf);
    const uint32_t sp = fw ? spf : spr, d = fw ? sb - sa : sa - sb;
    if (sp) { best = make_key(d, time_ms_dev(d, sp)); bc = fw ? 0 : 1; }
  }
  if (spf && lab0 != kKeyInf) { const unsigned long long k = lab0 + make_key(sb, b1.z); if (k < best) { best = k; bc = 2; } }
  if (spr && lab1 != kKeyInf) { const unsigned long long k = lab1 + make_key(L - sb, b1.w); if (k < best) { best = k; bc = 3; } }
  if (combo) *combo = bc;
  return best;
}

template <class Label>
__device__ __forceinline__ unsigned long long route_key(const Label& label, const uint4& a0, const uint4& b0,
                                                        const uint4& b1, int* combo) {
  const unsigned long long lab0 = d_spf(b0) ? label(b1.x) : kKeyInf;
  const unsigned long long lab1 = d_spr(b0) ? label(b1.y) : kKeyInf;
  return route_key_vals(a0, b0, b1, lab0, lab1, combo);
}

// root keys of a source candidate's two exits (forward to node1, reverse to node0)
__device__ __forceinline__ void exit_keys(const uint4& a0, uint32_t bound, unsigned long long& rk1,
                                          unsigned long long& rk0) {
  const uint32_t s = a0.y, L = a0.z, spf = d_spf(a0), spr = d_spr(a0);
  rk1 = (spf && L - s <= bound) ? make_key(L - s, time_ms_dev(L - s, spf)) : kKeyInf;
  rk0 = (spr && s <= bound) ? make_key(s, time_ms_dev(s, spr)) : kKeyInf;
}

// ------------------------------------------------------------------------------------------
// Bounded search shared by the wave tiers of K2 (routes) and of the path kernel.
template <int H, bool PATH>
struct SearchSmem {
  using FIdx = typename std::conditional<(H >= 65536), uint32_t, uint16_t>::type;
  uint32_t key[H];                 // (source << 28) | node
  unsigned long long lab[H];       // u64 (dist cm, time ms) key
  FIdx fa[H], fb[H];               // frontier (slot ids), ping-pong
  uint32_t inq[(H + 31) / 32];     // in-frontier bits (one word per 32 slots)
  uint32_t pred[PATH ? H : 1];
  uint32_t nf, nn, used, ovf;
};

// frontier membership bits: set returns true when this call set it (the slot joins the frontier)
__device__ __forceinline__ bool inq_set(uint32_t* inq, uint32_t slot) {
  const uint32_t bit = 1u << (slot & 31);
  return (atomicOr(&inq[slot >> 5], bit) & bit) == 0u;
}
__device__ __forceinline__ void inq_clear(uint32_t* inq, uint32_t slot) { atomicAnd(&inq[slot >> 5], ~(1u << (slot & 31))); }

template <int H, bool PATH>
__device__ __forceinline__ int h_insert(SearchSmem<H, PATH>& sm, uint32_t key) {
  uint32_t h = (key * 2654435761u) & (H - 1);
  for (int probe = 0; probe < H; ++probe) {
    uint32_t cur = sm.key[h];
    if (cur == key) return (int)h;
    if (cur == kEmpty) {
      cur = atomicCAS(&sm.key[h], kEmpty, key);
      if (cur == kEmpty) {
        if (atomicAdd(&sm.used, 1u) >= (uint32_t)(H * 3 / 4)) sm.ovf = 1u;
        return (int)h;
      }
      if (cur == key) return (int)h;
    }
    h = (h + 1) & (H - 1);
  }
  sm.ovf = 1u;
  return -1;
}

template <int H, bool PATH>
__device__ __forceinline__ int h_find(const SearchSmem<H, PATH>& sm, uint32_t key) {
  uint32_t h = (key * 2654435761u) & (H - 1);
  for (int probe = 0; probe < H; ++probe) {
    const uint32_t cur = sm.key[h];
    if (cur == key) return (int)h;
    if (cur == kEmpty) return -1;
    h = (h + 1) & (H - 1);
  }
  return -1;
}

template <int H, bool PATH>
__device__ __forceinline__ unsigned long long h_label(const SearchSmem<H, PATH>& sm, uint32_t key) {
  const int h = h_find(sm, key);
  return h < 0 ? kKeyInf : sm.lab[h];
}

// Frontier compaction: the active lanes of one wave instruction reserve their slots with ONE
// atomic by the lowest active lane (ballot -> popcount), which broadcasts the base by shuffle;
// each lane's slot is base + the number of active lanes below it.  Callable in divergent code.
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter) {
  const unsigned long long m = __ballot(1);
  const int lane = (int)(threadIdx.x & (kWave - 1));
  const int leader = __builtin_ctzll(m);
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
  base = (uint32_t)__shfl((int)base, leader, kWave);
  return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

template <int H, bool PATH>
struct HashLabel {
  const SearchSmem<H, PATH>& sm;
  uint32_t srcbits;
  __device__ unsigned long long operator()(uint32_t node) const { return h_label(sm, srcbits | node); }
};
// the same for walks that name a node with its road and side (single-source searches)
template <int H, bool PATH>
struct HashPathLabel {
  const SearchSmem<H, PATH>& sm;
  __device__ unsigned long long operator()(uint32_t node, uint32_t, uint32_t) const { return h_label(sm, node); }
};

// Early termination (round 4).  A search that serves known targets (a K2
// item's K_B target candidates, a path's chosen target) stops as soon as their route keys are
// final: at a round boundary every frontier label is >= F (the frontier minimum), and a node whose
// label is < F is final (its shortest path runs through nodes of smaller keys, all expanded), so a
// target whose current route key is < F can no longer improve.  When every target is below F the
// rest of the ball (up to the pair's bound, typically 4-5x the targets' distance at 30 s sampling)
// is never explored.  Strict <: a path's canonical predecessors (tight in-edges) of a node below F
// are then all final and in the hash, exactly as in the full search.
// `delta` (cm, kNone = off) limits a round to frontier nodes with keys <= F + delta; the others
// wait in the frontier (label-correcting rounds in near-Dijkstra order: fewer nodes re-relaxed and
// fewer touched beyond the targets).
struct SearchTargets {
  const uint4* tg;     // the targets' descriptors (global, 2 x uint4 each); null: none
  uint32_t n;          // how many (<= 64)
  uint32_t delta;      // cm, kNone: every frontier node every round
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The LDS search runs with W lanes per search: W = 64, one search per wave (a one-wave block:
// __syncthreads), or W = 16, four searches per wave (each group of 16 lanes on its own LDS
// slice; group steps are ordered by wave_sync, ballots masked to the group).
template <int W>
__device__ __forceinline__ void grp_sync() {
  if constexpr (W == kWave) __syncthreads();
  else wave_sync();
}
template <int W>
__device__ __forceinline__ int grp_lane() { return (int)(threadIdx.x & (W - 1)); }
template <int W>
__device__ __forceinline__ int grp_base() { return (int)(threadIdx.x & (kWave - 1) & ~(W - 1)); }
template <int W>
__device__ __forceinline__ unsigned long long grp_ballot(bool x) {
  const unsigned long long m = __ballot(x);
  if constexpr (W == kWave) return m;
  else return (m >> grp_base<W>()) & ((1ull << W) - 1ull);
}
// wave_append for a group: one atomic per group and instruction
template <int W>
__device__ __forceinline__ uint32_t grp_append(uint32_t* counter) {
  if constexpr (W == kWave) {
    return wave_append(counter);
  } else {
    const unsigned long long m = grp_ballot<W>(true);
    const int j = grp_lane<W>();
    const int leader = __builtin_ctzll(m);
    uint32_t base = 0;
    if (j == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, grp_base<W>() + leader, kWave);
    return base + (uint32_t)__popcll(m & ((1ull << j) - 1ull));
  }
}
template <int W>
__device__ __forceinline__ unsigned long long grp_min_u64(unsigned long long v) {
#pragma unroll
  for (int d = W / 2; d >= 1; d >>= 1) {
    const unsigned long long o = ((unsigned long long)(uint32_t)__shfl_xor((int)(v >> 32), d, W) << 32) |
                                 (uint32_t)__shfl_xor((int)(uint32_t)v, d, W);
    v = o < v ? o : v;
  }
  return v;
}

// Exact lexicographic shortest (dist, time) keys from the exits of n_src source
// candidates (descriptors src[0..n_src), source ids 0..n_src-1) to every node within
// `bound` cm, by synchronous label-correcting rounds over an LDS frontier compacted by ballot
// (wave_append).  All 64 lanes call it.
// With src == nullptr the single root is node `root` at key 0 (route-ball build).
// With targets (n_src == 1), the search may stop early: labels below the final frontier minimum
// are exact, the others are upper bounds (see SearchTargets).
template <int H, bool PATH, int W = kWave>
__device__ void bounded_search(SearchSmem<H, PATH>& sm, const DevGraph& g, int mode, uint32_t bound,
                               const uint4* src, uint32_t n_src, uint32_t root = 0,
                               SearchTargets tgt = SearchTargets{nullptr, 0u, kNone}) {
  using FIdx = typename SearchSmem<H, PATH>::FIdx;
  constexpr FIdx kDeferred = (FIdx)~(FIdx)0;
  static_assert((uint64_t)H <= (uint64_t)kDeferred, "frontier index needs a spare value");
  static_assert(W == kWave || W == 16, "64 or 16 lanes per search");
  const int lane = grp_lane<W>();
  const uint32_t acc = mode_access(mode);
  for (int h = lane; h < H; h += W) {
    sm.key[h] = kEmpty; sm.lab[h] = kKeyInf;
    if ((h & 31) == 0) sm.inq[h >> 5] = 0u;
    if (PATH) sm.pred[h] = kNone;
  }
  if (lane == 0) { sm.nf = 0; sm.nn = 0; sm.used = 0; sm.ovf = 0; }
  // targets: lane j holds target j's descriptor
  const bool has_tg = tgt.tg != nullptr && tgt.n != 0u;
  uint4 t0 = make_uint4(0u, 0u, 0u, 0u), t1 = t0;
  if (has_tg && (uint32_t)lane < tgt.n) { t0 = tgt.tg[2 * lane]; t1 = tgt.tg[2 * lane + 1]; }
  const bool use_min = has_tg || tgt.delta != kNone;
  grp_sync<W>();
  if (!src) {
    if (lane == 0) {
      const int slot = h_insert(sm, root);
      sm.lab[slot] = 0ull;
      sm.inq[slot >> 5] |= 1u << (slot & 31);
      sm.fa[sm.nf++] = (FIdx)slot;
    }
  } else if ((uint32_t)lane < 2u * n_src) {  // roots: two exits per source
    const uint32_t i = lane >> 1;
    const uint4 a0 = src[2 * i], a1 = src[2 * i + 1];
    unsigned long long rk1, rk0;
    exit_keys(a0, bound, rk1, rk0);
    const unsigned long long kk = (lane & 1) ? rk0 : rk1;
    if (kk != kKeyInf) {
      const uint32_t node = (lane & 1) ? a1.x : a1.y;
      const int slot = h_insert(sm, (i << 28) | node);
      if (slot >= 0) {
        const unsigned long long old = atomicMin(&sm.lab[slot], kk);
        if (kk < old && inq_set(sm.inq, slot)) sm.fa[grp_append<W>(&sm.nf)] = (FIdx)slot;
      }
    }
  }
  grp_sync<W>();
  const uint4 sa0 = src ? src[0] : make_uint4(0u, 0u, 0u, 0u);
  for (int round = 0;; ++round) {
    const uint32_t nf = sm.nf;
    if (nf == 0 || sm.ovf) break;
    if (round > 4 * H) { if (lane == 0) sm.ovf = 2u; break; }
    FIdx* cur = (round & 1) ? sm.fb : sm.fa;
    FIdx* nxt = (round & 1) ? sm.fa : sm.fb;
    unsigned long long thr = kKeyInf;
    if (use_min) {
      unsigned long long fm = kKeyInf;
      for (uint32_t q = lane; q < nf; q += W) {
        const unsigned long long l = sm.lab[cur[q]];
        fm = l < fm ? l : fm;
      }
      fm = grp_min_u64<W>(fm);
      if (has_tg) {   // every target's route key below the frontier minimum: final
        bool done = true;
        if ((uint32_t)lane < tgt.n) done = route_key(HashLabel<H, PATH>{sm, 0u}, sa0, t0, t1, nullptr) < fm;
        if (grp_ballot<W>(!done) == 0ull) break;
      }
      if (tgt.delta != kNone) thr = fm + ((unsigned long long)tgt.delta << 32);
    }
    if (thr == kKeyInf) {
      for (uint32_t q = lane; q < nf; q += W) inq_clear(sm.inq, cur[q]);
    } else {
      for (uint32_t q = lane; q < nf; q += W) {
        const FIdx slot = cur[q];
        if (sm.lab[slot] > thr) {   // waits for a later round (stays queued)
          nxt[grp_append<W>(&sm.nn)] = slot;
          cur[q] = kDeferred;
        } else {
          inq_clear(sm.inq, slot);
        }
      }
    }
    grp_sync<W>();
    for (uint32_t q = lane; q < nf; q += W) {
      const FIdx fs = cur[q];
      if (fs == kDeferred) continue;
      const int slot = fs;
      const uint32_t kk = sm.key[slot];
      const uint32_t node = kk & 0x0fffffffu, srcbits = kk & 0xf0000000u;
      const unsigned long long lab = sm.lab[slot];
      const uint32_t e0 = g.node_off[node], e1 = g.node_off[node + 1];
      for (uint32_t e = e0; e < e1; ++e) {
        const uint4 rec = g.edges[e];
        if (!edge_ok(rec.z, acc)) continue;
        const unsigned long long nk = lab + edge_key(rec, mode);
        if (key_dist(nk) > bound) continue;
        const int t = h_insert(sm, srcbits | rec.x);
        if (t < 0) continue;
        const unsigned long long old = atomicMin(&sm.lab[t], nk);
        if (nk < old && inq_set(sm.inq, (uint32_t)t)) nxt[grp_append<W>(&sm.nn)] = (FIdx)t;
      }
    }
    grp_sync<W>();
    if (lane == 0) { sm.nf = sm.nn; sm.nn = 0; }
    grp_sync<W>();
  }
  grp_sync<W>();
}

// ------------------------------------------------------------------------------------------
// Lane tiers: one lane runs one whole bounded Dijkstra.  Most searches settle a handful
// of nodes, so a wave-wide search would waste 60 lanes and pay LDS init + barriers.
// Edges are read as per-mode relax records {target, len_cm | kNoLen, time_ms, target's
// CSR range}: a settled node's label already holds its out-edge range, so each settle is
// ONE dependent round trip (the node's edge records), not two (offsets, then edges).
// Labels live in registers (kLaneCap slots, the common case; kTier2Cap in the second tier);
// keys are exact, so every store agrees.
#ifndef RM_LANE_CAP
#define RM_LANE_CAP 7
#endif
constexpr int kLaneCap = RM_LANE_CAP;
#ifndef RM_LANE_WPE
#define RM_LANE_WPE 4   // waves per SIMD the register lane tiers are compiled for
#endif
constexpr uint32_t kNoLen = 0xffffffffu;

template <int CAP>
struct RegLabelsT {
  static constexpr int kLaneCap = CAP;
  uint32_t node[CAP], rng[CAP], par[CAP];
  unsigned long long key[CAP];
  uint32_t n, settled;
  bool ovf;
  __device__ __forceinline__ void init() { n = 0; settled = 0; ovf = false; }
  __device__ __forceinline__ unsigned long long label(uint32_t v) const {
    unsigned long long k = kKeyInf;
#pragma unroll
    for (int x = 0; x < kLaneCap; ++x)
      if (x < (int)n && node[x] == v) k = key[x];
    return k;
  }
  __device__ __forceinline__ void relax(uint32_t v, unsigned long long k, uint32_t r, uint32_t from) {
    bool found = false;
#pragma unroll
    for (int x = 0; x < kLaneCap; ++x)
      if (x < (int)n && node[x] == v) {
        found = true;
        if (k < key[x]) { key[x] = k; par[x] = from; }
      }
    if (found) return;
    if (n >= (uint32_t)kLaneCap) { ovf = true; return; }
#pragma unroll
    for (int x = 0; x < kLaneCap; ++x)
      if (x == (int)n) { node[x] = v; key[x] = k; rng[x] = r; par[x] = from; }
    n++;
  }
  // settle the unsettled label with the smallest key; false when none is left.  `from`
  // is the settled node that gave it its final key (kNone for a root).
  __device__ __forceinline__ bool pick(unsigned long long& bk, uint32_t& r, uint32_t& u, uint32_t& from) {
    int bi = -1;
    bk = kKeyInf;
#pragma unroll
    for (int x = 0; x < kLaneCap; ++x)
      if (x < (int)n && !((settled >> x) & 1u) && key[x] < bk) { bk = key[x]; bi = x; r = rng[x]; u = node[x]; from = par[x]; }
    if (bi < 0) return false;
    settled |= 1u << bi;
    return true;
  }
};
using RegLabels = RegLabelsT<kLaneCap>;

template <class L>
struct StoreLabel {
  const L& s;
  __device__ unsigned long long operator()(uint32_t node) const { return s.label(node); }
};

struct NoStop {
  template <class L>
  __device__ bool operator()(const L&, unsigned long long) { return false; }
};
// a path search's single target: done once its route key is below the next settled key (labels
// below it are final, and so are the tight predecessors of such a label: see SearchTargets)
struct StopAtTarget {
  uint4 a0, b0, b1;
  template <class L>
  __device__ bool operator()(const L& S, unsigned long long bk) {
    return route_key(StoreLabel<L>{S}, a0, b0, b1, nullptr) < bk;
  }
};

// a K2 item's K_B targets: done once every target's route key is below the next settled key.
// Keys only fall, so a finite maximum stays an upper bound and is computed once; while some
// target is unreached it is recomputed every fourth settle.
constexpr uint32_t kStopMinBoundCm = 50000;   // pair bounds from which tier 2 stops at its targets
struct StopAtTargets {
  const uint4* tg;   // the pair's target descriptors (2 x uint4 each)
  uint32_t n;
  uint4 a0;
  unsigned long long kmax;
  uint32_t calls;
  template <class L>
  __device__ bool operator()(const L& S, unsigned long long bk) {
    if (!n) return false;   // no targets given: never stops
    if (kmax != kKeyInf && kmax != 0ull) return kmax < bk;
    if (kmax == kKeyInf && (++calls & 3u)) return false;
    unsigned long long m = 0ull;
    for (uint32_t j = 0; j < n && m != kKeyInf; ++j) {
      const unsigned long long k = route_key(StoreLabel<L>{S}, a0, tg[2 * j], tg[2 * j + 1], nullptr);
      m = k > m ? k : m;
    }
    kmax = m == 0ull ? 1ull : m;   // 0 marks "not computed yet"
    return m < bk;
  }
};

// bounded Dijkstra from the exits of the candidate described by (a0, a1); `stop(S, k)` is asked
// before each settle (k = the key about to be settled) and ends the search when true
template <class L, class Stop = NoStop>
__device__ __forceinline__ void lane_search(L& S, const DevGraph& g, const uint4* E, uint32_t bound,
                                            const uint4& a0, const uint4& a1, unsigned long long& rk1,
                                            unsigned long long& rk0, Stop stop = Stop{}) {
  S.init();
  exit_keys(a0, bound, rk1, rk0);
  const uint32_t r1 = rk1 != kKeyInf ? g.node_rng[a1.y] : 0u;
  const uint32_t r0 = rk0 != kKeyInf ? g.node_rng[a1.x] : 0u;
  if (rk1 != kKeyInf) S.relax(a1.y, rk1, r1, kNone);
  if (rk0 != kKeyInf) S.relax(a1.x, rk0, r0, kNone);
  unsigned long long bk;
  uint32_t r = 0, u = 0, from = kNone;
  while (S.pick(bk, r, u, from)) {
    if (stop(S, bk)) break;
    const uint32_t e0 = r >> 5, deg = r & 31u;
    for (uint32_t q0 = 0; q0 < deg; q0 += 4) {
      uint4 rec[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) rec[x] = E[e0 + min(q0 + x, deg - 1u)];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        // an edge back to the settled node that gave u its key can never improve it
        if (q0 + x >= deg || rec[x].y == kNoLen || rec[x].x == from) continue;
        const unsigned long long nk = bk + make_key(rec[x].y, rec[x].z);
        if (key_dist(nk) <= bound) S.relax(rec[x].x, nk, rec[x].w, u);
      }
    }
    if (S.ovf) break;
  }
}

// routes from source a0 to the KB targets of pair slot p; results staged in LDS
// (res[j * stride]) and stored after the last load (a store before a load-use costs a
// full round trip: gfx9 loads and stores share vmcnt)
// labels for the path walk: label of node x, which is the `side` endpoint (0: node0,
// 1: node1) of `road` (the ball tier probes by road; the search tiers ignore both)
template <class L>
struct SearchPathLabels {
  const L& s;
  __device__ unsigned long long operator()(uint32_t x, uint32_t, uint32_t) const { return s.label(x); }
};

// Turn weight (rule 3b) of the route of combination `combo` from source (a0, a1) to target
// (b0, b1) in a search with labels `lab` (exit root keys rk1 / rk0): the canonical path walked back
// from the entry node as the path stage walks it, one turn per node, the exit node's arriving edge
// being the source road in the exit's direction.  0 for the direct combinations; ok false when a
// predecessor is missing (not reached for a valid route).
template <class PL>
__device__ __forceinline__ uint32_t search_turn_walk(const DevGraph& g, const PL& lab, int mode, const uint4& a0,
                                                     const uint4& a1, const uint4& b0, const uint4& b1,
                                                     unsigned long long rk1, unsigned long long rk0, int combo, bool& ok) {
  ok = true;
  if (combo < 2) return 0u;
  const uint32_t acc = mode_access(mode);
  const uint32_t side = combo == 2 ? 0u : 1u;
  uint32_t hs = head_start(g.road_head[b0.x], side);   // the entry edge leaves its node with this heading
  uint32_t x = side ? b1.y : b1.x;
  unsigned long long lx = lab(x, b0.x, side);
  const uint32_t hwa = g.road_head[a0.x];
  uint32_t U = 0;
  for (uint32_t guard = 0; guard < (1u << 20); ++guard) {
    if (lx == kKeyInf) break;
    if (x == a1.y && lx == rk1) return U + g.turn_w[turn_degree(head_back(hwa, 0u), hs)];   // exit forward: node1
    if (x == a1.x && lx == rk0) return U + g.turn_w[turn_degree(head_back(hwa, 1u), hs)];   // exit reverse: node0
    bool found = false;
    uint4 rec = make_uint4(0u, 0u, 0u, 0u);
    unsigned long long plu = kKeyInf;
    for (uint32_t q = g.in_off[x], q1 = g.in_off[x + 1]; q < q1; ++q) {
      const uint4 r = g.in_rec[q];
      const uint32_t inf = g.in_info[q];
      if (!edge_ok(inf, acc)) continue;
      const unsigned long long lu = lab(r.y, r.z >> 1, r.z & 1u);
      if (lu != kKeyInf && lu + make_key(r.w, time_ms_dev(r.w, mode_speed_dkph(mode, inf & 0xffffu))) == lx) {
        rec = r; plu = lu; found = true;
        break;
      }
    }
    if (!found) break;
    const uint32_t hw = g.road_head[rec.z >> 1], rev = rec.z & 1u;
    U += g.turn_w[turn_degree(head_back(hw, rev), hs)];
    hs = head_start(hw, rev);
    x = rec.y;
    lx = plu;
  }
  ok = false;
  return 0u;
}

// the turn weights of a search's routes (rule 3b): what search_turn_walk needs besides the labels
struct TurnCtx {
  uint4 a1;                      // the source's second descriptor word (its road's endpoints)
  unsigned long long rk1, rk0;   // exit root keys
  int mode;
  bool on;                       // the pair has turn costs (pair_info.w) and the batch a route_d array
  uint32_t factor;               // pair_info.w
  double gc;                     // the pair's measurement distance
};

template <class Label, class PL>
__device__ __forceinline__ void route_targets(const DevGraph& g, const DevBatch& b, const Label& lab, const PL& plab,
                                              const uint4& a0, uint64_t p, uint32_t KB, uint32_t bound, uint32_t tmax,
                                              uint64_t ob, uint32_t* res, int stride, const TurnCtx& tc) {
  const uint64_t brow = p * kMaxCand * 2;
  for (uint32_t j0 = 0; j0 < KB; j0 += 4) {
    uint4 t0[4], t1[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const uint32_t jc = min(j0 + x, KB - 1u);
      t0[x] = b.cand_desc[brow + 2 * jc];
      t1[x] = b.cand_desc[brow + 2 * jc + 1];
    }
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      int combo = -1;
      const unsigned long long key = route_key(lab, a0, t0[x], t1[x], &combo);
      uint32_t r = kRouteInvalid;
      if (key != kKeyInf && key_dist(key) <= bound && key_time(key) <= tmax) r = key_dist(key);
      res[((j0 + x) & (kMaxCand - 1)) * stride] = r;
      if (tc.on && j0 + x < KB) {   // a batch with turn costs (rare in a search tier): stored straight away
        bool ok = true;
        const uint32_t u = (r == kRouteInvalid || !tc.factor)
                               ? 0u
                               : search_turn_walk(g, plab, tc.mode, a0, tc.a1, t0[x], t1[x], tc.rk1, tc.rk0, combo, ok);
        if (!ok) trace_fail(b, p, kErrRounds);
        b.route_d[ob + j0 + x] = route_term(r, u, tc.factor, tc.gc);
      }
    }
  }
  for (uint32_t j = 0; j < KB; ++j) b.route[ob + j] = res[j * stride];
}

// ------------------------------------------------------------------------------------------
// K2 ball tier (balls.hpp): when the pair's bound fits in the mode's ball radius, the
// source's bounded search is replaced by table probes: label(v) = min over the exits x of
// rk_x + key(x -> v).  Both exits' first probes of a target are issued together; collisions
// continue by linear probing (tables are at most half full, so an empty slot ends it).
// A table is keyed by road, so one probe per exit gives the labels of both entry nodes.
constexpr uint32_t kBallMaxKeys = kBallMaxKeysHost;

// row of `road` in a node's table (balls.hpp), continuing the probe from first-probe row e
// (rmask: the road-id bits of the row's first word, rm_common.hpp ball_road_mask)
__device__ __forceinline__ uint4 ball_resolve(const uint4* ent, const uint2& h, uint32_t road, uint4 e, uint32_t rmask) {
  if ((e.x & rmask) == road || e.x == kNone) return e;
  const uint32_t mask = (1u << h.y) - 1u;
  uint32_t s = ball_slot(road, h.y);
  for (;;) {
    s = (s + 1u) & mask;
    e = ent[ball_row0(h.x) + s];
    if ((e.x & rmask) == road || e.x == kNone) return e;
  }
}

// ball_resolve that also gives the row's slot (s: the first probe's slot on entry)
__device__ __forceinline__ uint4 ball_resolve_at(const uint4* ent, const uint2& h, uint32_t road, uint4 e, uint32_t rmask,
                                                 uint32_t& s) {
  if ((e.x & rmask) == road || e.x == kNone) return e;
  const uint32_t mask = (1u << h.y) - 1u;
  for (;;) {
    s = (s + 1u) & mask;
    e = ent[ball_row0(h.x) + s];
    if ((e.x & rmask) == road || e.x == kNone) return e;
  }
}

// keys from a row (kKeyInf for an endpoint outside the ball or a road not in the table)
__device__ __forceinline__ unsigned long long row_key0(const uint4& e) { return ball_key0(e.x, e.y, e.w); }
__device__ __forceinline__ unsigned long long row_key1(const uint4& e) { return ball_key1(e.x, e.z, e.w); }

__device__ __forceinline__ unsigned long long ball_label(unsigned long long rk1, unsigned long long d1,
                                                         unsigned long long rk0, unsigned long long d0) {
  unsigned long long k = kKeyInf;
  if (d1 != kKeyInf) k = rk1 + d1;
  if (d0 != kKeyInf && rk0 + d0 < k) k = rk0 + d0;
  return k;
}

#ifndef RM_BALL_WPE
#define RM_BALL_WPE 4
#endif
// K2 ball tier, block-expanded (round 3).  A block takes 256 consecutive (pair, source) items,
// whose routes form one contiguous range of b.route.  Phase 1, one lane per item: the pair's
// constants, the source's exit keys and both exits' table headers go to LDS, and the item's
// lanes of the range are marked in an owner map.  Phase 2 deals the range over the lanes, one
// (source, target) transition per lane and step: the target's descriptor, both exits' probes of
// the target road, the label, the key, one coalesced store.  No lane walks a target loop of its
// own (the round-2 kernel's lanes ran to their wave's largest K_B, each target two dependent
// round trips after the last), and two transitions per lane are in flight at once.
#ifndef RM_K2_ITEMS
#define RM_K2_ITEMS 256
#endif
constexpr int kK2Items = RM_K2_ITEMS;   // (pair, source) items per block
constexpr int kK2Threads = 256;         // threads per block (phase 2: one transition per thread and step)
static_assert(kK2Items <= kK2Threads && kK2Items % 64 == 0, "phase 1 runs one item per thread");
// graphs from this many nodes take the locality order by default (Engine::locality_default),
// and so do batches sampled this sparsely on average (Matcher::run)
constexpr uint64_t kLocalityNodes = 150000;
constexpr double kLocalitySparseS = 10.0;
// global-address-space 16-byte pointer: loads through it are global_load_dwordx4 even when the
// address went through LDS (a generic pointer there would become a flat load)
typedef unsigned int k2_v4 __attribute__((ext_vector_type(4)));
typedef const k2_v4 __attribute__((address_space(1)))* k2_gptr;
__device__ __forceinline__ uint4 k2_ld(k2_gptr p) {
  const k2_v4 v = *p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
// A source item in full (k_turn_walks rebuilds it for the walked turn weights, k2_route_turn)
struct K2Src {
  unsigned long long ent;        // the item's mode's table rows (a global address: see k2_gptr)
  uint2 h1, h0;                  // table headers of the exits (bits 0: no table)
  unsigned long long rk1, rk0;   // exit root keys (kKeyInf: that exit is unusable)
  uint32_t road, s;              // source road and offset on it (direct combinations)
  uint32_t bound, tmax;          // pair bounds; bound = kNone: handed to the search tiers
  uint32_t lim;                  // routes with distance <= lim are exact from the tables (ball_exact_limit)
};
// per item of a batch with turn costs (rule 3b): the mode's turn rows, the source road's headings
// and endpoints, the pair's factor
struct K2Turn {
  unsigned long long trn;        // turn rows of the item's mode (a global address)
  uint32_t hw;                   // heading word of the source road (rm_common.hpp head_back)
  uint32_t fac;                  // pair_info.w: the factor's float bits; 0: the item has no turn costs
  uint32_t n0, n1;               // the source road's endpoints (the exits' nodes)
  uint32_t mode, pad;
};
// The item record of the kernel without turn costs, 60 bytes (round 6).  LDS sets this kernel's
// occupancy: at 80 bytes per item (22.8 -> 24.9 KB per block) C2's K2 went 0.866 -> 0.935 ms with
// the same loop (6 blocks of 4 waves per CU instead of 7); at 60 bytes a block fits 20 KB and a CU
// holds 8 of them.  The mode's table base comes from a per-mode LDS table (the road word's top
// bits), the root keys are split into words (4-byte alignment), and the descriptor and route
// offsets are folded with the item's first transition (dbase, obase).
struct K2SrcS {
  uint32_t dbase;                // transition q of the block reads descriptor pair dbase + q
  uint32_t obase;                // ... and writes b.route[obase + q]
  uint32_t h1x, h1y, h0x, h0y;   // table headers of the exits (uint2 would align to 8)
  uint32_t rk1l, rk1h, rk0l, rk0h;   // exit root keys, split
  uint32_t roadm;                // source road | mode << 29
  uint32_t s, bound, tmax, lim;
};
static_assert(sizeof(K2SrcS) == 60, "K2SrcS is 60 bytes");
// walked turn weights (ties between the exits) a K2 block lists for k_turn_walks: each goes to the
// block's own region of b.walk (an LDS counter, the count written first at the block's end; no
// global atomics: 639 k appends per C2 step to one counter took K2 with turn costs from 1.5 to 3.1
// ms); past kWalkPerBlock they are marked in place for k_turn_walks_marked
constexpr uint32_t kWalkPerBlock = 512;
constexpr uint32_t kRouteWalk = 0xfffffffeu;   // (a route left to k_turn_walks_marked)
template <bool TURN>
struct K2Smem {
  K2SrcS src[kK2Items];
  unsigned long long ent_mode[5];      // each mode's table rows (a mode without tables: a dummy array)
  unsigned long long trn_mode[TURN ? 5 : 1];   // ... and turn rows
  uint8_t owner[kK2Items * kMaxCand];   // transition of the block -> item of the block
  uint32_t wsum[kK2Threads / 64];
  uint32_t redo[kK2Items / 32];         // bit o: a route of item o was not exact from the tables
  uint16_t tw16[TURN ? kTurnDegrees + 1 : 2];  // the turn weights (DevGraph::turn_w; k2_turn_weight)
  uint32_t wn;                            // (with turn costs) the block's walked turn weights
};
// (both records fit 20 KB per block with turn costs too: 8 blocks per CU)
template <class SM>
__device__ __forceinline__ void k2_redo(SM& sm, uint32_t o) { atomicOr(&sm.redo[o >> 5], 1u << (o & 31u)); }

// Bounds beyond the ball radius (round 4).  A table holds every node within R of its exit, so a
// node absent from exit x's table is more than R away from it and any route through it is longer
// than rk_x + R.  A route key computed from the tables is therefore exact whenever its distance
// is <= rk_x + R for every usable exit x -- whatever the pair's bound: the shorter routes all run
// inside the tables, and (for the path stage) so do the canonical predecessors of every node on
// them.  Items whose routes all pass are answered by the tables; the others go to the search
// tiers.  With bound <= R the limit is never needed (every route within the bound is in the
// tables): kNone.
__device__ __forceinline__ uint32_t ball_exact_limit(uint32_t bound, uint32_t radius, unsigned long long rk1,
                                                     unsigned long long rk0) {
  if (bound <= radius) return kNone;
  uint32_t lim = kNone;
  if (rk1 != kKeyInf) lim = min(lim, key_dist(rk1) + radius);
  if (rk0 != kKeyInf) lim = min(lim, key_dist(rk0) + radius);
  // a route the tables miss is longer than lim: beyond the bound too when lim >= bound, so
  // every result (valid or not) is the tables'
  return lim >= bound ? kNone : lim;
}

// route of item S to the target described by (t0, t1), from the target road's rows (r1, r0)
// in the tables of S's two exits (kRouteInvalid when there is none within the bounds); `exact`
// false when the tables cannot decide it (ball_exact_limit)
__device__ __forceinline__ uint32_t k2_route_v(unsigned long long rk1, unsigned long long rk0, uint32_t road, uint32_t s,
                                               uint32_t lim, uint32_t bound, uint32_t tmax, const uint4& t0,
                                               const uint4& t1, const uint4& r1, const uint4& r0, bool& exact) {
  const unsigned long long lab0 = ball_label(rk1, row_key0(r1), rk0, row_key0(r0));
  const unsigned long long lab1 = ball_label(rk1, row_key1(r1), rk0, row_key1(r0));
  const uint4 a0 = make_uint4(road, s, 0u, 0u);   // route_key_vals reads the source's road and offset
  const unsigned long long key = route_key_vals(a0, t0, t1, lab0, lab1, nullptr);
  exact = lim == kNone || (key != kKeyInf && key_dist(key) <= lim);
  return (key != kKeyInf && key_dist(key) <= bound && key_time(key) <= tmax) ? key_dist(key) : kRouteInvalid;
}
__device__ __forceinline__ uint32_t k2_route(const K2Src& S, const uint4& t0, const uint4& t1, const uint4& r1,
                                             const uint4& r0, bool& exact) {
  return k2_route_v(S.rk1, S.rk0, S.road, S.s, S.lim, S.bound, S.tmax, t0, t1, r1, r0, exact);
}

// labels from the route balls of the two exits (see k_routes_ball2)
struct BallPathLabels {
  const uint4* ent;
  uint2 h1, h0;
  unsigned long long rk1, rk0;
  uint32_t rm;   // road-id bits of a row's first word
  // both exits' rows of `road` (a dummy row for an unusable exit), first probes issued together
  __device__ void rows(uint32_t road, uint4& r1, uint4& r0) const {
    // both first probes issued together: an unusable exit reads row 0 (valid: the mode has
    // tables) and its row is replaced by the empty row afterwards
    const bool u1 = rk1 != kKeyInf, u0 = rk0 != kKeyInf;
    const uint64_t i1 = u1 ? ball_row0(h1.x) + ball_slot(road, h1.y) : 0u;
    const uint64_t i0 = u0 ? ball_row0(h0.x) + ball_slot(road, h0.y) : 0u;
    const uint4 l1 = ent[i1], l0 = ent[i0];
    const uint4 none = make_uint4(kNone, kBallNoDist, kBallNoDist, 0u);
    r1 = ball_resolve(ent, h1, road, u1 ? l1 : none, rm);
    r0 = ball_resolve(ent, h0, road, u0 ? l0 : none, rm);
  }
  __device__ unsigned long long operator()(uint32_t, uint32_t road, uint32_t side) const {
    uint4 r1, r0;
    rows(road, r1, r0);
    return side ? ball_label(rk1, row_key1(r1), rk0, row_key1(r0)) : ball_label(rk1, row_key0(r1), rk0, row_key0(r0));
  }
};

// One step of the ball-tier walk back from node x (label lx, rows r1/r0 of a road with x at
// `side`): x's canonical predecessor in the two-exit search.  Where exactly one exit gives x
// its label, the tight in-edges of the two-exit search are that exit's own and the canonical
// one is the predecessor stored in its row; on a tie between the exits they are the union of
// both, and the canonical one the smaller stored index (in_rec is in edge-id order).  Only
// when that index was not stored (7 or more in-edges before it) are the in-edges scanned.
// Returns false when no predecessor exists (not reached for a valid route).
__device__ __forceinline__ bool ball_pred_step(const DevGraph& g, const BallPathLabels& lab, uint32_t acc, int mode,
                                               uint32_t x, unsigned long long lx, const uint4& r1, const uint4& r0,
                                               uint32_t side, uint4& rec, unsigned long long& plu) {
  const uint32_t q0 = g.in_off[x];
  const unsigned long long k1 = side ? row_key1(r1) : row_key0(r1), k0 = side ? row_key1(r0) : row_key0(r0);
  uint32_t idx = kBallPredNone;
  if (lab.rk1 != kKeyInf && k1 != kKeyInf && lab.rk1 + k1 == lx) idx = min(idx, ball_pred(r1.x, side, lab.rm));
  if (lab.rk0 != kKeyInf && k0 != kKeyInf && lab.rk0 + k0 == lx) idx = min(idx, ball_pred(r0.x, side, lab.rm));
  if (idx < kBallPredNone) {
    rec = g.in_rec[q0 + idx];
    plu = kKeyInf;   // the caller reads the predecessor's label from its rows
    return true;
  }
  for (uint32_t q = q0, q1 = g.in_off[x + 1]; q < q1; ++q) {
    const uint4 r = g.in_rec[q];
    const uint32_t inf = g.in_info[q];
    if (!edge_ok(inf, acc)) continue;
    const unsigned long long lu = lab(r.y, r.z >> 1, r.z & 1u);
    if (lu != kKeyInf && lu + make_key(r.w, time_ms_dev(r.w, mode_speed_dkph(mode, inf & 0xffffu))) == lx) {
      rec = r;
      plu = lu;
      return true;
    }
  }
  return false;
}

// Turn weight of a route the tables answer, by walking its two-exit canonical path back through
// the tables (ball_pred_step, as the path stage walks): for the routes whose turn row cannot give it
// -- a tie between the exits at the entry node (the canonical path may mix both exits' trees: a
// source at a node whose route runs along its own road ties there), or a row without its sum.
// x: the entry node (at `side` of road rb), r1 / r0: both exits' rows of rb.  ok false: no path.
__device__ uint32_t ball_turn_walk(const DevGraph& g, const BallPathLabels& lab, const K2Turn& T, uint32_t rb,
                                   uint32_t x, uint32_t side, uint4 r1, uint4 r0, bool& ok) {
  const uint32_t acc = mode_access((int)T.mode);
  uint32_t hs = head_start(g.road_head[rb], side);
  unsigned long long lx = side ? ball_label(lab.rk1, row_key1(r1), lab.rk0, row_key1(r0))
                               : ball_label(lab.rk1, row_key0(r1), lab.rk0, row_key0(r0));
  uint32_t U = 0;
  ok = true;
  for (uint32_t guard = 0; guard <= 2u * kBallMaxKeysHost + 2u; ++guard) {
    if (lx == kKeyInf) break;
    if (x == T.n1 && lx == lab.rk1) return U + g.turn_w[turn_degree(head_back(T.hw, 0u), hs)];
    if (x == T.n0 && lx == lab.rk0) return U + g.turn_w[turn_degree(head_back(T.hw, 1u), hs)];
    uint4 rec;
    unsigned long long plu;
    if (!ball_pred_step(g, lab, acc, (int)T.mode, x, lx, r1, r0, side, rec, plu)) break;
    const uint32_t hw = g.road_head[rec.z >> 1], rev = rec.z & 1u;
    U += g.turn_w[turn_degree(head_back(hw, rev), hs)];
    hs = head_start(hw, rev);
    x = rec.y;
    side = rev;   // the edge's start: node0 of its road when it runs forward
    lab.rows(rec.z >> 1, r1, r0);
    lx = side ? ball_label(lab.rk1, row_key1(r1), lab.rk0, row_key1(r0))
              : ball_label(lab.rk1, row_key0(r1), lab.rk0, row_key0(r0));
  }
  ok = false;
  return 0u;
}

// A route the tables answer in a batch with turn costs (rule 3b, TURN), and its distance term
// d = turn_m + |route_m - gc| (route_term).  The turn weight: when one exit gives the entry node
// its label strictly, that exit's turn row holds the weight of the path from the exit node on and
// the heading it leaves the exit node with, and the turn at the exit node is from the source road;
// otherwise (a tie, or a row without its sum) ball_turn_walk.
// pt1 / pt0: both exits' turn rows at the first-probe slots h1s / h0s, loaded with the probes (a
// route resolved past a collision reloads its row); tw: the turn weights in LDS
__device__ __forceinline__ uint32_t k2_route_turn(const DevGraph& g, const K2Src& S, const K2Turn& T, const uint4& t0,
                                                  const uint4& t1, const uint4& r1, const uint4& r0, uint32_t s1,
                                                  uint32_t s0, uint32_t h1s, uint32_t h0s, const uint2& pt1,
                                                  const uint2& pt0, const uint32_t* tw, double gc, bool& exact, double& d) {
  const unsigned long long k10 = row_key0(r1), k00 = row_key0(r0), k11 = row_key1(r1), k01 = row_key1(r0);
  const unsigned long long l10 = k10 != kKeyInf ? S.rk1 + k10 : kKeyInf, l00 = k00 != kKeyInf ? S.rk0 + k00 : kKeyInf;
  const unsigned long long l11 = k11 != kKeyInf ? S.rk1 + k11 : kKeyInf, l01 = k01 != kKeyInf ? S.rk0 + k01 : kKeyInf;
  const unsigned long long lab0 = l00 < l10 ? l00 : l10, lab1 = l01 < l11 ? l01 : l11;
  const uint4 a0 = make_uint4(S.road, S.s, 0u, 0u);
  int combo = -1;
  const unsigned long long key = route_key_vals(a0, t0, t1, lab0, lab1, &combo);
  exact = S.lim == kNone || (key != kKeyInf && key_dist(key) <= S.lim);
  const bool valid = key != kKeyInf && key_dist(key) <= S.bound && key_time(key) <= S.tmax;
  uint32_t U = 0u;
  if (T.fac && valid && combo >= 2 && exact) {
    const uint32_t side = (uint32_t)combo - 2u;
    const unsigned long long la = side ? l11 : l10, lb = side ? l01 : l00;
    uint32_t w = kTurnNone;
    const bool e1 = la < lb;
    if (la != lb) {
      uint2 trow = e1 ? pt1 : pt0;
      if ((e1 ? s1 != h1s : s0 != h0s)) {   // resolved past a collision: the row of the final slot
        const uint64_t row = e1 ? ball_row0(S.h1.x) + s1 : ball_row0(S.h0.x) + s0;
        trow = reinterpret_cast<const uint2*>(T.trn)[row];
      }
      w = side ? trow.y : trow.x;
    }
    if ((w & kTurnTMask) != kTurnNone) {
      U = tw[turn_degree(head_back(T.hw, e1 ? 0u : 1u), w >> kTurnHeadShift)] + (w & kTurnTMask);
    } else {
      const BallPathLabels lab{(const uint4*)S.ent, S.h1, S.h0, S.rk1, S.rk0, g.ball_road_mask};
      bool ok = true;
      U = ball_turn_walk(g, lab, T, t0.x, side ? t1.y : t1.x, side, r1, r0, ok);
      if (!ok) exact = false;
    }
  }
  const uint32_t r = valid ? key_dist(key) : kRouteInvalid;
  d = route_term(r, U, T.fac, gc);
  return r;
}

// ---- k_routes_ball2 phase 2 (round 6, VERDICT r05 item 2: "take control of the waits").  A
// software-pipelined loop was built and measured: the probe addresses formed branch-free (every
// exit's header valid, ball_slot_bf), 24-byte descriptor reads, two register sets so a step issued
// its probes, then the next step's descriptors, then waited for its own probes only (the ISA
// checked: vmcnt(7)/(6) waits, no waits between the issue groups).  C2's K2 did not move (0.951 vs
// 0.931 ms for the unpipelined loop on the same build, bench-style timing): the kernel is not bound
// by where its waits sit but by occupancy and VALU (valu_frac 0.65).  What moved it was LDS: the
// item records at 80 bytes gave 6 blocks per CU, at 72 bytes 7 (0.935 -> 0.866 ms), at 60 (K2SrcS)
// 8.  The turn-cost kernel keeps the pipelined loop (k2_phase2_pipe_t).
typedef unsigned int k2_u2 __attribute__((ext_vector_type(2)));
typedef const k2_u2 __attribute__((address_space(1)))* k2_gptr2;
__device__ __forceinline__ uint2 k2_ld2(k2_gptr2 p) {
  const k2_u2 v = *p;
  return make_uint2(v.x, v.y);
}
// a row or the empty row, selected per word (a select of the aggregate went through scratch)
__device__ __forceinline__ uint4 k2_row_or_none(bool use, const uint4& e) {
  return make_uint4(use ? e.x : kNone, use ? e.y : kBallNoDist, use ? e.z : kBallNoDist, use ? e.w : 0u);
}
// ball_resolve through a global-address-space pointer
__device__ __forceinline__ uint4 ball_resolve_g(k2_gptr ent, const uint2& h, uint32_t road, uint4 e, uint32_t rmask) {
  if ((e.x & rmask) == road || e.x == kNone) return e;
  const uint32_t mask = (1u << h.y) - 1u;
  uint32_t s = ball_slot(road, h.y);
  for (;;) {
    s = (s + 1u) & mask;
    e = k2_ld(ent + (ball_row0(h.x) + s));
    if ((e.x & rmask) == road || e.x == kNone) return e;
  }
}
// phase 2 without turn costs: two transitions per lane and step, every load of a step issued before
// any is used (the descriptors unconditionally -- a handed-over item's descriptor is as valid an
// address --, the four first probes branch-free with an unused probe reading a valid dummy row)
__device__ __forceinline__ uint4 ball_resolve_at_g(k2_gptr ent, const uint2& h, uint32_t road, uint4 e, uint32_t rmask,
                                                   uint32_t& s) {
  if ((e.x & rmask) == road || e.x == kNone) return e;
  const uint32_t mask = (1u << h.y) - 1u;
  for (;;) {
    s = (s + 1u) & mask;
    e = k2_ld(ent + (ball_row0(h.x) + s));
    if ((e.x & rmask) == road || e.x == kNone) return e;
  }
}
// phase 2 without turn costs: 3 (default, round 6) one transition per lane and step with the next
// step's descriptor loaded ahead; 1 the same without the prefetch; 2 two transitions per step
#ifndef RM_K2_PLAIN_STEP
#define RM_K2_PLAIN_STEP 3
#endif
template <class SM>
__device__ __forceinline__ void k2_phase2_slim(SM& sm, const DevBatch& b, uint32_t n, uint32_t rm, k2_gptr dummy) {
  const uint4 none = make_uint4(kNone, kBallNoDist, kBallNoDist, 0u);
  if (RM_K2_PLAIN_STEP == 3) {   // one transition per step, the next step's descriptor loaded ahead
    // (its loads are in flight with this step's probes: one memory round trip per step instead of
    // two; 54 VGPRs, 8 waves per SIMD; C2 routes 0.782 -> 0.766 ms)
    uint32_t q = threadIdx.x;
    uint4 ta0 = make_uint4(0u, 0u, 0u, 0u);
    uint2 ta1 = make_uint2(0u, 0u);
    if (q < n) {
      const K2SrcS& A0 = sm.src[sm.owner[q]];
      const uint4* pd = b.cand_desc + 2 * (uint64_t)(A0.dbase + q);
      ta0 = k2_ld((k2_gptr)(const void*)pd);
      ta1 = k2_ld2((k2_gptr2)(const void*)(reinterpret_cast<const uint2*>(pd + 1) + 1));
    }
    for (; q < n; q += kK2Threads) {
      const K2SrcS& A = sm.src[sm.owner[q]];
      const uint32_t qn = q + kK2Threads < n ? q + kK2Threads : q;   // clamped: a valid address
      const K2SrcS& An = sm.src[sm.owner[qn]];
      const uint4* pdn = b.cand_desc + 2 * (uint64_t)(An.dbase + qn);
      const uint4 nt0 = k2_ld((k2_gptr)(const void*)pdn);
      const uint2 nt1 = k2_ld2((k2_gptr2)(const void*)(reinterpret_cast<const uint2*>(pdn + 1) + 1));
      const bool la = A.bound != kNone;
      const unsigned long long ak1 = (unsigned long long)A.rk1h << 32 | A.rk1l, ak0 = (unsigned long long)A.rk0h << 32 | A.rk0l;
      const bool ua = la && ta0.w != 0u;
      const bool ua1 = ua && ak1 != kKeyInf, ua0 = ua && ak0 != kKeyInf;
      const k2_gptr ea = (k2_gptr)(const void*)(uintptr_t)sm.ent_mode[A.roadm >> 29];
      const k2_gptr pa1 = ua1 ? ea + (ball_row0(A.h1x) + ball_slot(ta0.x, A.h1y)) : dummy;
      const k2_gptr pa0 = ua0 ? ea + (ball_row0(A.h0x) + ball_slot(ta0.x, A.h0y)) : dummy;
      const uint4 la1 = k2_ld(pa1), la0 = k2_ld(pa0);
      bool xa = true;
      const uint32_t r = k2_route_v(ak1, ak0, A.roadm & 0x1fffffffu, A.s, A.lim, A.bound, A.tmax, ta0,
                                    make_uint4(0u, 0u, ta1.x, ta1.y),
                                    ball_resolve_g(ea, make_uint2(A.h1x, A.h1y), ta0.x, k2_row_or_none(ua1, la1), rm),
                                    ball_resolve_g(ea, make_uint2(A.h0x, A.h0y), ta0.x, k2_row_or_none(ua0, la0), rm), xa);
      if (la) {
        b.route[A.obase + q] = r;
        if (!xa) k2_redo(sm, sm.owner[q]);
      }
      ta0 = nt0;
      ta1 = nt1;
    }
    return;
  }
  if (RM_K2_PLAIN_STEP == 1) {   // (A/B: one transition per lane and step, fewer registers)
    for (uint32_t q = threadIdx.x; q < n; q += kK2Threads) {
      const K2SrcS& A = sm.src[sm.owner[q]];
      const bool la = A.bound != kNone;
      const uint4* pda = b.cand_desc + 2 * (uint64_t)(A.dbase + q);
      const uint4 ta0 = k2_ld((k2_gptr)(const void*)pda);
      const uint2 ta1 = k2_ld2((k2_gptr2)(const void*)(reinterpret_cast<const uint2*>(pda + 1) + 1));
      const unsigned long long ak1 = (unsigned long long)A.rk1h << 32 | A.rk1l, ak0 = (unsigned long long)A.rk0h << 32 | A.rk0l;
      const bool ua = la && ta0.w != 0u;
      const bool ua1 = ua && ak1 != kKeyInf, ua0 = ua && ak0 != kKeyInf;
      const k2_gptr ea = (k2_gptr)(const void*)(uintptr_t)sm.ent_mode[A.roadm >> 29];
      const k2_gptr pa1 = ua1 ? ea + (ball_row0(A.h1x) + ball_slot(ta0.x, A.h1y)) : dummy;
      const k2_gptr pa0 = ua0 ? ea + (ball_row0(A.h0x) + ball_slot(ta0.x, A.h0y)) : dummy;
      const uint4 la1 = k2_ld(pa1), la0 = k2_ld(pa0);
      bool xa = true;
      const uint32_t r = k2_route_v(ak1, ak0, A.roadm & 0x1fffffffu, A.s, A.lim, A.bound, A.tmax, ta0,
                                    make_uint4(0u, 0u, ta1.x, ta1.y),
                                    ball_resolve_g(ea, make_uint2(A.h1x, A.h1y), ta0.x, k2_row_or_none(ua1, la1), rm),
                                    ball_resolve_g(ea, make_uint2(A.h0x, A.h0y), ta0.x, k2_row_or_none(ua0, la0), rm), xa);
      if (la) {
        b.route[A.obase + q] = r;
        if (!xa) k2_redo(sm, sm.owner[q]);
      }
    }
    return;
  }
  for (uint32_t q = threadIdx.x; q < n; q += 2 * kK2Threads) {
    const uint32_t qb = q + kK2Threads;
    const bool hb = qb < n;
    const uint32_t qB = hb ? qb : q;
    const K2SrcS& A = sm.src[sm.owner[q]];
    const K2SrcS& B = sm.src[sm.owner[qB]];
    const bool la = A.bound != kNone, lb = hb && B.bound != kNone;
    const uint4* pda = b.cand_desc + 2 * (uint64_t)(A.dbase + q);
    const uint4* pdb = b.cand_desc + 2 * (uint64_t)(B.dbase + qB);
    const uint4 ta0 = k2_ld((k2_gptr)(const void*)pda), tb0 = k2_ld((k2_gptr)(const void*)pdb);
    // of the second half only the entry times
    const uint2 ta1 = k2_ld2((k2_gptr2)(const void*)(reinterpret_cast<const uint2*>(pda + 1) + 1));
    const uint2 tb1 = k2_ld2((k2_gptr2)(const void*)(reinterpret_cast<const uint2*>(pdb + 1) + 1));
    const unsigned long long ak1 = (unsigned long long)A.rk1h << 32 | A.rk1l, ak0 = (unsigned long long)A.rk0h << 32 | A.rk0l;
    const unsigned long long bk1 = (unsigned long long)B.rk1h << 32 | B.rk1l, bk0 = (unsigned long long)B.rk0h << 32 | B.rk0l;
    const bool ua = la && ta0.w != 0u, ub = lb && tb0.w != 0u;   // some direction of the target road is usable
    const bool ua1 = ua && ak1 != kKeyInf, ua0 = ua && ak0 != kKeyInf;
    const bool ub1 = ub && bk1 != kKeyInf, ub0 = ub && bk0 != kKeyInf;
    const k2_gptr ea = (k2_gptr)(const void*)(uintptr_t)sm.ent_mode[A.roadm >> 29];
    const k2_gptr eb = (k2_gptr)(const void*)(uintptr_t)sm.ent_mode[B.roadm >> 29];
    const k2_gptr pa1 = ua1 ? ea + (ball_row0(A.h1x) + ball_slot(ta0.x, A.h1y)) : dummy;
    const k2_gptr pa0 = ua0 ? ea + (ball_row0(A.h0x) + ball_slot(ta0.x, A.h0y)) : dummy;
    const k2_gptr pb1 = ub1 ? eb + (ball_row0(B.h1x) + ball_slot(tb0.x, B.h1y)) : dummy;
    const k2_gptr pb0 = ub0 ? eb + (ball_row0(B.h0x) + ball_slot(tb0.x, B.h0y)) : dummy;
    const uint4 la1 = k2_ld(pa1), la0 = k2_ld(pa0), lb1 = k2_ld(pb1), lb0 = k2_ld(pb0);
    bool xa = true, xb = true;
    if (la)
      b.route[A.obase + q] = k2_route_v(ak1, ak0, A.roadm & 0x1fffffffu, A.s, A.lim, A.bound, A.tmax, ta0,
                                        make_uint4(0u, 0u, ta1.x, ta1.y),
                                        ball_resolve_g(ea, make_uint2(A.h1x, A.h1y), ta0.x, k2_row_or_none(ua1, la1), rm),
                                        ball_resolve_g(ea, make_uint2(A.h0x, A.h0y), ta0.x, k2_row_or_none(ua0, la0), rm), xa);
    if (lb)
      b.route[B.obase + qb] = k2_route_v(bk1, bk0, B.roadm & 0x1fffffffu, B.s, B.lim, B.bound, B.tmax, tb0,
                                         make_uint4(0u, 0u, tb1.x, tb1.y),
                                         ball_resolve_g(eb, make_uint2(B.h1x, B.h1y), tb0.x, k2_row_or_none(ub1, lb1), rm),
                                         ball_resolve_g(eb, make_uint2(B.h0x, B.h0y), tb0.x, k2_row_or_none(ub0, lb0), rm), xb);
    if (!xa) k2_redo(sm, sm.owner[q]);
    if (!xb) k2_redo(sm, sm.owner[qB]);
  }
  (void)none;
}

// k_routes_ball2<true>'s two-per-step loop (round 6): the route of a transition from the tables,
// and what its turn weight needs -- nothing (U = 0: no turn costs, an invalid or direct route, a
// route the tables cannot decide), the turn row of the exit that strictly gives the entry node its
// label (`row`, read after the probes), or the walk (a tie between the exits).  The same decisions
// as k2_route_turn.
struct K2TurnKey {
  uint64_t row;      // need 1: the turn row's index (the winning exit's final slot)
  uint32_t r;        // route cm or kRouteInvalid
  uint32_t need;     // 0: U = 0, 1: from the row, 2: walk
  uint32_t side;     // entry at node1 (combo 3)
  uint32_t e1;       // the winning exit is the forward one (node1)
  bool exact;
};
__device__ __forceinline__ K2TurnKey k2_turn_key(const K2SrcS& S, unsigned long long rk1, unsigned long long rk0,
                                                 uint32_t fac, const uint4& t0, const uint4& t1, const uint4& r1,
                                                 const uint4& r0, uint32_t s1, uint32_t s0) {
  const unsigned long long k10 = row_key0(r1), k00 = row_key0(r0), k11 = row_key1(r1), k01 = row_key1(r0);
  const unsigned long long l10 = k10 != kKeyInf ? rk1 + k10 : kKeyInf, l00 = k00 != kKeyInf ? rk0 + k00 : kKeyInf;
  const unsigned long long l11 = k11 != kKeyInf ? rk1 + k11 : kKeyInf, l01 = k01 != kKeyInf ? rk0 + k01 : kKeyInf;
  const unsigned long long lab0 = l00 < l10 ? l00 : l10, lab1 = l01 < l11 ? l01 : l11;
  const uint4 a0 = make_uint4(S.roadm & 0x1fffffffu, S.s, 0u, 0u);
  int combo = -1;
  const unsigned long long key = route_key_vals(a0, t0, t1, lab0, lab1, &combo);
  K2TurnKey k;
  k.exact = S.lim == kNone || (key != kKeyInf && key_dist(key) <= S.lim);
  const bool valid = key != kKeyInf && key_dist(key) <= S.bound && key_time(key) <= S.tmax;
  k.r = valid ? key_dist(key) : kRouteInvalid;
  k.need = 0u;
  k.side = combo == 3 ? 1u : 0u;
  const unsigned long long la = k.side ? l11 : l10, lb = k.side ? l01 : l00;
  k.e1 = la < lb ? 1u : 0u;
  k.row = k.e1 ? ball_row0(S.h1x) + s1 : ball_row0(S.h0x) + s0;
  if (fac && valid && combo >= 2 && k.exact) k.need = la != lb ? 1u : 2u;
  return k;
}
// the turn weight U from the winner's turn row (wx, wy: its node0 / node1 words), or kNone when
// it must be walked (a tie, or a row without its sum)
// (tw16: the turn weights in 16 bits, the U-turn's 65536 stored as 0 -- K2's LDS budget)
__device__ __forceinline__ uint32_t k2_turn_weight(const K2TurnKey& k, uint32_t hw, uint32_t wx, uint32_t wy,
                                                   const uint16_t* tw16) {
  if (k.need == 0u) return 0u;
  const uint32_t w = k.side ? wy : wx;
  if (k.need == 2u || (w & kTurnTMask) == kTurnNone) return kNone;
  const uint32_t d = turn_degree(head_back(hw, k.e1 ? 0u : 1u), w >> kTurnHeadShift);
  return (d == 0u ? 65536u : (uint32_t)tw16[d]) + (w & kTurnTMask);
}

// phase 2 with turn costs (round 6): one transition per lane and step, with both exits' turn rows
// read with the probes at their first-probe slots (no dependent third load; a row resolved past a
// collision -- rare -- reloads its turn row).  The item records are the plain kernel's (the source
// road's heading word, the pair's factor and gc come from global memory with the descriptor), so the
// block fits 20 KB of LDS and a CU holds 8.  A route whose turn weight needs the walk (a tie between
// the exits, a row without its sum: 1.3 % of C2's transitions) goes to a list that k_turn_walks
// walks right after this kernel, one lane each: the walk's registers (86 VGPRs with it in this
// loop, 60 without) stay out of this kernel.
typedef unsigned int k2_v2 __attribute__((ext_vector_type(2)));
typedef const k2_v2 __attribute__((address_space(1)))* k2_trow;
template <class SM>
__device__ __forceinline__ void k2_phase2_turn1(const DevGraph& g, SM& sm, const DevBatch& b, uint32_t n, uint32_t rm,
                                                k2_gptr dummy, uint32_t t0i) {
  const k2_trow tdummy = (k2_trow)(const void*)b.cand_desc;
  for (uint32_t q = threadIdx.x; q < n; q += kK2Threads) {
    const uint32_t o = sm.owner[q];
    const K2SrcS& A = sm.src[o];
    const bool la = A.bound != kNone;
    const uint32_t di = A.dbase + q;   // = pair * 16 + target
    const uint32_t p = di >> 4;
    const uint4* pda = b.cand_desc + 2 * (uint64_t)di;
    const uint4 ta0 = k2_ld((k2_gptr)(const void*)pda);
    const uint2 ta1 = k2_ld2((k2_gptr2)(const void*)(reinterpret_cast<const uint2*>(pda + 1) + 1));
    const uint32_t road = A.roadm & 0x1fffffffu;
    const uint32_t fac = b.pair_info[p].w, hw = g.road_head[road];
    const double gc = b.gc[p];
    const unsigned long long ak1 = (unsigned long long)A.rk1h << 32 | A.rk1l, ak0 = (unsigned long long)A.rk0h << 32 | A.rk0l;
    const bool ua = la && ta0.w != 0u;
    const bool ua1 = ua && ak1 != kKeyInf, ua0 = ua && ak0 != kKeyInf;
    const uint32_t mode = A.roadm >> 29;
    const k2_gptr ea = (k2_gptr)(const void*)(uintptr_t)sm.ent_mode[mode];
    const k2_trow tra = (k2_trow)(const void*)(uintptr_t)sm.trn_mode[mode];
    const uint32_t h1s = ball_slot(ta0.x, A.h1y), h0s = ball_slot(ta0.x, A.h0y);
    const uint64_t i1 = ball_row0(A.h1x) + h1s, i0 = ball_row0(A.h0x) + h0s;
    const uint4 la1 = k2_ld(ua1 ? ea + i1 : dummy), la0 = k2_ld(ua0 ? ea + i0 : dummy);
    // (a pair without turn costs may be of a mode without turn rows: no row read)
    const k2_v2 v1 = *(ua1 && fac ? tra + i1 : tdummy), v0 = *(ua0 && fac ? tra + i0 : tdummy);
    uint32_t s1 = h1s, s0 = h0s;
    const uint4 r1 = ball_resolve_at_g(ea, make_uint2(A.h1x, A.h1y), ta0.x, k2_row_or_none(ua1, la1), rm, s1);
    const uint4 r0 = ball_resolve_at_g(ea, make_uint2(A.h0x, A.h0y), ta0.x, k2_row_or_none(ua0, la0), rm, s0);
    const K2TurnKey k = k2_turn_key(A, ak1, ak0, fac, ta0, make_uint4(0u, 0u, ta1.x, ta1.y), r1, r0, s1, s0);
    k2_v2 w = k.e1 ? v1 : v0;
    if (k.need == 1u && (k.e1 ? s1 != h1s : s0 != h0s)) w = tra[k.row];   // resolved past a collision
    const uint32_t U = k2_turn_weight(k, hw, w.x, w.y, sm.tw16);
    if (!la) continue;
    if (U != kNone) {
      b.route[A.obase + q] = k.r;
      b.route_d[A.obase + q] = route_term(k.r, U, fac, gc);
      if (!k.exact) k2_redo(sm, o);
    } else {   // walked by k_turn_walks (item << 4 | target); a full list: the search tiers take the item
      const uint32_t item = t0i + o;
      const uint32_t x = atomicAdd(&sm.wn, 1u);
      if (x < kWalkPerBlock && item < (1u << 28)) {
        b.walk[(uint64_t)blockIdx.x * (kWalkPerBlock + 1) + 1 + x] = item << 4 | (di & 15u);
      } else {   // marked in place for k_turn_walks_marked
        b.route[A.obase + q] = kRouteWalk;
        b.route_d[A.obase + q] = __longlong_as_double((long long)((unsigned long long)item << 4 | (di & 15u)));
        b.ctl[15] = 1u;
      }
    }
  }
}

// The turn weights K2 left to walk (each K2 block's region of b.walk), one lane each: the item again as
// k_routes_ball2's phase 1 forms it, the route with both exits' turn rows at their first-probe
// slots, and the walk through the tables (k2_route_turn / ball_turn_walk).  A route the tables
// cannot decide hands its item to the search tiers, which run next.
// one walked turn weight: item t's route to its pair's target j (ro: its route index, known to the
// marker scan; kNone: from the item)
__device__ void k2_walk_one(const DevGraph& g, const DevBatch& b, uint32_t t, uint32_t j) {
  const uint32_t rm = g.ball_road_mask;
  const k2_gptr dummy = (k2_gptr)(const void*)b.cand_desc;
  const k2_trow tdummy = (k2_trow)(const void*)b.cand_desc;
  const uint32_t p = b.src_item[t];
  const uint4 pi = b.pair_info[p];
  const uint32_t i = t - b.src_off[p];
  const uint32_t KB = (pi.z >> 8) & 0xffu;
  const uint64_t ro = (uint64_t)b.trans_off[p] + i * KB + j;
  const uint64_t arow = ((uint64_t)(p - 1) * kMaxCand + i) * 2;
  const uint4 a0 = b.cand_desc[arow], a1 = b.cand_desc[arow + 1];
  const int mode = (int)(pi.z >> 16);
  K2Src A;
  exit_keys(a0, pi.x, A.rk1, A.rk0);
  A.lim = ball_exact_limit(pi.x, g.ball_radius[mode], A.rk1, A.rk0);
  const uint2* hp = g.ball_hdr[mode];
  A.h1 = A.rk1 != kKeyInf ? hp[a1.y] : make_uint2(0u, 1u);
  A.h0 = A.rk0 != kKeyInf ? hp[a1.x] : make_uint2(0u, 1u);
  A.ent = (unsigned long long)(uintptr_t)g.ball_ent[mode];
  A.road = a0.x;
  A.s = a0.y;
  A.bound = pi.x;
  A.tmax = pi.y;
  K2Turn T;
  T.fac = pi.w;
  T.trn = (unsigned long long)(uintptr_t)g.ball_turn[mode];
  T.hw = g.road_head[a0.x];
  T.n0 = a1.x;
  T.n1 = a1.y;
  T.mode = (uint32_t)mode;
  T.pad = 0u;
  const k2_gptr da = (k2_gptr)(const void*)(b.cand_desc + 2 * ((uint64_t)p * kMaxCand + j));
  const uint4 ta0 = k2_ld(da), ta1 = k2_ld(da + 1);
  const double gc = b.gc[p];
  const bool ua = ta0.w != 0u;
  const bool ua1 = ua && A.rk1 != kKeyInf, ua0 = ua && A.rk0 != kKeyInf;
  const uint32_t h1s = ball_slot(ta0.x, A.h1.y), h0s = ball_slot(ta0.x, A.h0.y);
  const uint64_t i1 = ball_row0(A.h1.x) + h1s, i0 = ball_row0(A.h0.x) + h0s;
  const k2_gptr ea = (k2_gptr)(const void*)(uintptr_t)A.ent;
  const k2_trow tra = (k2_trow)(const void*)(uintptr_t)T.trn;
  const uint4 la1 = k2_ld(ua1 ? ea + i1 : dummy), la0 = k2_ld(ua0 ? ea + i0 : dummy);
  const k2_v2 v1 = *(ua1 && T.fac ? tra + i1 : tdummy), v0 = *(ua0 && T.fac ? tra + i0 : tdummy);
  uint32_t s1 = h1s, s0 = h0s;
  const uint4 r1 = ball_resolve_at_g(ea, A.h1, ta0.x, k2_row_or_none(ua1, la1), rm, s1);
  const uint4 r0 = ball_resolve_at_g(ea, A.h0, ta0.x, k2_row_or_none(ua0, la0), rm, s0);
  bool ok = true;
  double d = 0.0;
  b.route[ro] = k2_route_turn(g, A, T, ta0, ta1, r1, r0, s1, s0, h1s, h0s, make_uint2(v1.x, v1.y),
                              make_uint2(v0.x, v0.y), g.turn_w, gc, ok, d);
  b.route_d[ro] = d;
  if (!ok) b.rl_routes_0[atomicAdd(&b.ctl[1], 1u)] = t;
}
// (launched with K2's grid and n_arg, one block per K2 block: the block's region of b.walk)
#ifndef RM_WALK_THREADS
#define RM_WALK_THREADS 64
#endif
constexpr uint32_t kWalkThreads = RM_WALK_THREADS;
__global__ void __launch_bounds__(kWalkThreads) k_turn_walks(DevGraph g, DevBatch b, uint32_t n_arg) {
  if (steady_abort(b)) return;
  const uint32_t n_items = n_arg != kNone ? n_arg : (uint32_t)b.tot[1];
  const uint32_t nblk = (uint32_t)(((uint64_t)n_items + kK2Items - 1) / kK2Items);
  if (blockIdx.x >= nblk) return;
  const uint32_t* reg = b.walk + (uint64_t)blockIdx.x * (kWalkPerBlock + 1);
  const uint32_t nw = reg[0];
  for (uint32_t e = threadIdx.x; e < nw; e += blockDim.x) {
    const uint32_t wv = reg[1 + e];
    k2_walk_one(g, b, wv >> 4, wv & 15u);
  }
}
constexpr uint32_t kWalkScanGrid = 2048;
// the walks a K2 block could not list (more than kWalkPerBlock): marked in place -- route
// kRouteWalk, route_d's bits the item and target -- and found by one scan of the routes, run only
// when some block overflowed (ctl[15])
__global__ void __launch_bounds__(256) k_turn_walks_marked(DevGraph g, DevBatch b) {
  if (steady_abort(b) || b.ctl[15] == 0u) return;
  const uint64_t n = b.tot[0];
  for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (uint64_t)gridDim.x * blockDim.x) {
    if (b.route[x] != kRouteWalk) continue;
    const unsigned long long wv = (unsigned long long)__double_as_longlong(b.route_d[x]);
    k2_walk_one(g, b, (uint32_t)(wv >> 4), (uint32_t)(wv & 15u));
  }
}

// (without turn costs 7 waves per SIMD: the slim records' 20 KB of LDS per block allow 8 blocks per
// CU, but 8 waves squeeze the loop into 64 VGPRs with 24 bytes of spills per lane -- C2's K2 0.947
// ms; at 7 waves (72 VGPRs, no spills) 0.835 ms, 6: 0.837, round 5's kernel 0.866)
#ifndef RM_BALL_WPE_PLAIN
#define RM_BALL_WPE_PLAIN 8
#endif
template <bool TURN>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TURN ? RM_BALL_WPE : RM_BALL_WPE_PLAIN))) k_routes_ball2(DevGraph g, DevBatch b, uint32_t n_arg) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  __shared__ K2Smem<TURN> sm;
  // kNone: a small run's launch, sized by the upper bound; the item count is on the device
  const uint32_t n_items = n_arg != kNone ? n_arg : (uint32_t)b.tot[1];
  // (blocks past the items' exit; the rest map onto XCDs by the item-block count, so a grid sized
  // from an upper bound still spreads the work over every XCD)
  const uint32_t nblk = (uint32_t)(((uint64_t)n_items + kK2Items - 1) / kK2Items);
  if (blockIdx.x >= nblk) return;
  const uint32_t t0i = xcd_block(blockIdx.x, nblk) * kK2Items;   // first item of the block
  const uint32_t t = t0i + threadIdx.x;
  const uint32_t tl = min(n_items, t0i + kK2Items) - 1u;              // last item of the block
  const bool live = threadIdx.x < (uint32_t)kK2Items && t <= tl;   // (items <= threads per block)
  // ---- phase 1: one lane per item
  uint32_t KB = 0, ob = 0, pq = 0, md = 0;
  K2Src S;
  if (threadIdx.x == 0) {   // each mode's table rows and turn rows (a mode without: a valid dummy array)
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      sm.ent_mode[m] = (unsigned long long)(uintptr_t)(g.ball_ent[m] ? (const void*)g.ball_ent[m] : (const void*)b.cand_desc);
      if constexpr (TURN)
        sm.trn_mode[m] = (unsigned long long)(uintptr_t)(g.ball_turn[m] ? (const void*)g.ball_turn[m] : (const void*)b.cand_desc);
    }
  }
  if (live) {
    const uint32_t p = b.src_item[t];
    pq = p;
    const uint4 pi = b.pair_info[p];
    const uint32_t i = t - b.src_off[p];
    KB = (pi.z >> 8) & 0xffu;
    ob = b.trans_off[p] + i * KB;
    const uint64_t arow = ((uint64_t)(p - 1) * kMaxCand + i) * 2;
    const uint4 a0 = b.cand_desc[arow], a1 = b.cand_desc[arow + 1];
    const int mode = (int)(pi.z >> 16);
    md = (uint32_t)mode;
    exit_keys(a0, pi.x, S.rk1, S.rk0);
    // the mode's tables answer any bound: beyond their radius, the routes they decide
    const bool fits = (g.ball_mask >> mode) & 1u;
    S.lim = ball_exact_limit(pi.x, g.ball_radius[mode], S.rk1, S.rk0);
    S.h1 = S.h0 = make_uint2(0u, 1u);
    if (fits) {   // both headers loaded together, then kept where the exit is usable
      const uint2* hp = g.ball_hdr[mode];
      const uint2 x1 = hp[a1.y], x0 = hp[a1.x];
      if (S.rk1 != kKeyInf) S.h1 = x1;
      if (S.rk0 != kKeyInf) S.h0 = x0;
    }
    S.road = a0.x;
    S.s = a0.y;
    S.bound = pi.x;
    S.tmax = pi.y;
    bool turn_ok = true;
    if constexpr (TURN) turn_ok = !pi.w || ((g.ball_turn_mask >> mode) & 1u);   // no turn rows: the search tiers weigh the turns
    if (!fits || S.h1.y == 0u || S.h0.y == 0u || !turn_ok) {   // the search tiers take it (they run later)
      S.bound = kNone;
      b.rl_routes_0[atomicAdd(&b.ctl[1], 1u)] = t;
    }
  }
  // the block's transitions: an exclusive scan of the items' K_B (in slot order the items' routes
  // are one contiguous range and this is ob - the first ob; in locality order they are not)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t incl = KB;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(incl, d, 64);
    if (lane >= d) incl += u;
  }
  if (lane == 63) sm.wsum[wv] = incl;
  __syncthreads();
  uint32_t wbase = 0, n = 0;
#pragma unroll
  for (int w = 0; w < kK2Threads / 64; ++w) {
    const uint32_t x = sm.wsum[w];
    wbase += w < wv ? x : 0u;
    n += x;
  }
  if (live) {
    const uint32_t rel = wbase + incl - KB;
    K2SrcS z;
    z.dbase = pq * kMaxCand - rel;
    z.obase = ob - rel;
    z.h1x = S.h1.x; z.h1y = S.h1.y;
    z.h0x = S.h0.x; z.h0y = S.h0.y;
    z.rk1l = (uint32_t)S.rk1; z.rk1h = (uint32_t)(S.rk1 >> 32);
    z.rk0l = (uint32_t)S.rk0; z.rk0h = (uint32_t)(S.rk0 >> 32);
    z.roadm = S.road | md << 29;
    z.s = S.s;
    z.bound = S.bound;
    z.tmax = S.tmax;
    z.lim = S.lim;
    sm.src[threadIdx.x] = z;
    for (uint32_t j = 0; j < KB; ++j) sm.owner[rel + j] = (uint8_t)threadIdx.x;
  }
  if (threadIdx.x < (uint32_t)kK2Items / 32) sm.redo[threadIdx.x] = 0;
  if constexpr (TURN) {
    if (threadIdx.x < (uint32_t)kTurnDegrees) sm.tw16[threadIdx.x] = (uint16_t)g.turn_w[threadIdx.x];   // (65536 -> 0)
    if (threadIdx.x == 0) sm.wn = 0u;
  }
  __syncthreads();
  // ---- phase 2: the block's routes, one transition per lane and step (k2_phase2_slim /
  // k2_phase2_turn1)
  const k2_gptr dummy = (k2_gptr)(const void*)b.cand_desc;
  const uint32_t rm = g.ball_road_mask;
  if constexpr (TURN) k2_phase2_turn1(g, sm, b, n, rm, dummy, t0i);
  if constexpr (!TURN) k2_phase2_slim(sm, b, n, rm, dummy);
  // items with a route the tables could not decide: the search tiers recompute all of its routes
  __syncthreads();
  if (live && ((sm.redo[threadIdx.x >> 5] >> (threadIdx.x & 31u)) & 1u) && sm.src[threadIdx.x].bound != kNone)
    b.rl_routes_0[atomicAdd(&b.ctl[1], 1u)] = t;
  if constexpr (TURN) {   // the count of the block's region of b.walk
    if (threadIdx.x == 0) b.walk[(uint64_t)blockIdx.x * (kWalkPerBlock + 1)] = min(sm.wn, kWalkPerBlock);
  }
}


// K2 lane tier: one lane per (layer pair, source) item.  The pair constants come from
// one dwordx4 (pair_info) and every candidate from its 32-byte descriptor.  A search
// that outgrows the registers is queued (as its item) for the LDS lane tier.
// With `listed`, thread q takes the q-th item the ball tier handed over (rl_routes_0, ctl[1]).
constexpr uint64_t kListedGrid = 4096;   // blocks of a grid-stride launch over hand-over lists

// TURN: compiled with the turn-weight walks (rule 3b) only for batches with turn costs (they
// cost the plain tier registers: scratch 12 -> 64 bytes per lane)
template <bool TURN>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RM_LANE_WPE))) k_routes_lane(DevGraph g, DevBatch b, uint32_t n_items, int listed) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  // grid-stride: a listed launch is sized for every item but usually finds few hand-overs
  const uint32_t n = listed ? b.ctl[1] : (n_items != kNone ? n_items : (uint32_t)b.tot[1]);
  __shared__ uint32_t s_res[kMaxCand][256];
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
  const uint32_t t = listed ? b.rl_routes_0[q] : q;
  const uint32_t p = b.src_item[t];
  const uint4 pi = b.pair_info[p];
  const uint32_t i = t - b.src_off[p];
  const uint32_t base = b.trans_off[p];
  const uint32_t bound = pi.x, tmax = pi.y, KB = (pi.z >> 8) & 0xffu;
  const int mode = (int)(pi.z >> 16);
  const uint64_t arow = ((uint64_t)(p - 1) * kMaxCand + i) * 2;
  const uint4 a0 = b.cand_desc[arow], a1 = b.cand_desc[arow + 1];
  RegLabels S;
  unsigned long long rk1, rk0;
  // no early stop here: at the bounds this tier completes (tens of metres) the targets' check
  // costs more than the settles it saves (C2 --ball-radius 0: 2.1 -> 3.4 ms); tier 2 has it
  lane_search(S, g, g.relax[mode], bound, a0, a1, rk1, rk0);
  if (S.ovf) {
    b.rl_routes_a[atomicAdd(&b.ctl[3], 1u)] = t;
    continue;
  }
  route_targets(g, b, StoreLabel<RegLabels>{S}, SearchPathLabels<RegLabels>{S}, a0, p, KB, bound, tmax,
                (uint64_t)base + i * KB, &s_res[0][threadIdx.x], 256, TurnCtx{a1, rk1, rk0, mode, TURN, pi.w, TURN ? b.gc[p] : 0.0});
  }
}

// K2 second register tier: the items the first tier queued, RM_TIER2_CAP labels per lane
// (compiled for fewer waves per SIMD); what still overflows goes to the wave tier.
#ifndef RM_TIER2_CAP
#define RM_TIER2_CAP 12
#endif
constexpr int kTier2Cap = RM_TIER2_CAP;
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) k_routes_reg2(DevGraph g, DevBatch b) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  __shared__ uint32_t s_res[kMaxCand][256];
  const uint32_t n_items = b.ctl[3];
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n_items; q += gridDim.x * blockDim.x) {
    const uint32_t t = b.rl_routes_a[q];
    const uint32_t p = b.src_item[t];
    const uint4 pi = b.pair_info[p];
    const uint32_t i = t - b.src_off[p];
    const uint32_t base = b.trans_off[p];
    const uint32_t bound = pi.x, tmax = pi.y, KB = (pi.z >> 8) & 0xffu;
    const int mode = (int)(pi.z >> 16);
    const uint64_t arow = ((uint64_t)(p - 1) * kMaxCand + i) * 2;
    const uint4 a0 = b.cand_desc[arow], a1 = b.cand_desc[arow + 1];
    RegLabelsT<kTier2Cap> S;
    unsigned long long rk1, rk0;
    // the early stop pays from bounds of a few blocks (C3's 30 s pairs); at 1 Hz bounds its
    // checks cost more than they save (C2 --ball-radius 0: 0.69 -> 1.0 ms)
    lane_search(S, g, g.relax[mode], bound, a0, a1, rk1, rk0,
                StopAtTargets{b.cand_desc + (uint64_t)p * kMaxCand * 2, bound >= kStopMinBoundCm ? KB : 0u, a0, 0ull, 0u});
    if (S.ovf) {
      const uint32_t x = atomicAdd(&b.ctl[5], 1u);
      b.rl_routes_b[x] = t;
      continue;
    }
    route_targets(g, b, StoreLabel<RegLabelsT<kTier2Cap>>{S}, SearchPathLabels<RegLabelsT<kTier2Cap>>{S}, a0, p, KB,
                  bound, tmax, (uint64_t)base + i * KB, &s_res[0][threadIdx.x], 256,
                  TurnCtx{a1, rk1, rk0, mode, b.route_d != nullptr, pi.w, b.route_d ? b.gc[p] : 0.0});
  }
}

// path of one chosen transition (slot p) with a lane-resident search: canonical
// predecessors (smallest-id tight in-edge from a labelled node) walked back from the
// entry node.  Returns false when the search outgrew its label store (caller queues p).
// Canonical predecessor of node x (label lx): the smallest-id usable in-edge (u -> x) with
// label(u) + key(edge) == lx, in ascending edge id.  Each in-edge is one self-contained record
// (edge, source node, road|rev, length; info word): one round trip before its label probe
// instead of three dependent loads (in_edge -> edges -> edge_src).  Probing several in-edges
// at once was slower: most nodes find the tight edge first, and the extra probes and
// registers cost more than the overlap (C2 paths 0.32 -> 0.39 ms).
template <class PL>
__device__ __forceinline__ bool find_pred(const DevGraph& g, const PL& lab, uint32_t acc, int mode, uint32_t x,
                                          unsigned long long lx, uint32_t& pe, uint32_t& pu, unsigned long long& plu) {
  for (uint32_t q = g.in_off[x], q1 = g.in_off[x + 1]; q < q1; ++q) {
    const uint4 r = g.in_rec[q];
    const uint32_t inf = g.in_info[q];
    if (!edge_ok(inf, acc)) continue;
    // r.y is the edge's start: node0 of its road when the edge runs forward
    const unsigned long long lu = lab(r.y, r.z >> 1, r.z & 1u);
    if (lu != kKeyInf && lu + make_key(r.w, time_ms_dev(r.w, mode_speed_dkph(mode, inf & 0xffffu))) == lx) {
      pe = r.x; pu = r.y; plu = lu;
      return true;
    }
  }
  return false;
}

// Walk the chosen transition's route back from its entry node by canonical predecessors
// (smallest-id usable in-edge from a labelled node whose label + edge key equals the
// node's label) and write its edges.  `key`/`combo` are the transition's route key and
// combination (route_key_vals).
template <class PL>
__device__ __forceinline__ void path_walk(const DevGraph& g, const DevBatch& b, uint64_t p, const PL& lab, int mode,
                                          const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1,
                                          unsigned long long rk1, unsigned long long rk0, unsigned long long key,
                                          int combo, int cap) {
  const uint32_t acc = mode_access(mode);
  const uint32_t n1a = a1.y, n0a = a1.x;
  uint32_t* inl = b.path_inline + p * kInlinePath;
  if (combo <= 1) {
    b.route_dist[p] = key_dist(key);
    b.path_sab[p] = make_uint2(a0.y, b0.y);
    inl[0] = combo == 0 ? g.road_fwd[a0.x] : g.road_rev[a0.x];
    b.path_cnt[p] = 1;
    b.path_off[p] = 0;
    return;
  }
  // walk back from the entry node.  Edges are shifted into registers (front = travel
  // order) and stored after the walk: a store inside the walk would make every following
  // load wait for it (shared vmcnt).
  const uint32_t entry_e = combo == 2 ? g.road_fwd[b0.x] : g.road_rev[b0.x];
  const uint32_t v0 = combo == 2 ? b1.x : b1.y;
  uint32_t n = 1, x = v0;
  unsigned long long lx = lab(v0, b0.x, combo == 2 ? 0u : 1u);
  uint32_t pr[kInlinePath];
#pragma unroll
  for (int q = 0; q < kInlinePath; ++q) pr[q] = entry_e;
  for (int guard = 0;; ++guard) {
    if (lx == kKeyInf || guard > cap) { trace_fail(b, p, kErrRounds); return; }
    if ((x == n1a && lx == rk1) || (x == n0a && lx == rk0)) break;
    uint32_t pe = kNone, pu = 0;
    unsigned long long plu = kKeyInf;
    if (!find_pred(g, lab, acc, mode, x, lx, pe, pu, plu)) { trace_fail(b, p, kErrRounds); return; }
#pragma unroll
    for (int q = kInlinePath - 1; q > 0; --q) pr[q] = pr[q - 1];
    pr[0] = pe;
    ++n;
    x = pu;
    lx = plu;
  }
  const uint32_t exit_e = (x == n1a) ? g.road_fwd[a0.x] : g.road_rev[a0.x];
#pragma unroll
  for (int q = kInlinePath - 1; q > 0; --q) pr[q] = pr[q - 1];
  pr[0] = exit_e;
  ++n;
  b.route_dist[p] = key_dist(key);
  b.path_sab[p] = make_uint2(a0.y, b0.y);
  b.path_cnt[p] = n;
  if (n <= (uint32_t)kInlinePath) {
#pragma unroll
    for (int q = 0; q < kInlinePath; ++q)
      if ((uint32_t)q < n) inl[q] = pr[q];
    b.path_off[p] = 0;
    return;
  }
  // long path: pool slot, second walk writing in travel order
  const uint32_t at = atomicAdd(&b.ctl[0], n);
  if ((uint64_t)at + n > b.path_cap) { atomicOr(&b.ctl[2], kErrPathOverflow); b.path_off[p] = kNone; return; }
  b.path_off[p] = at;
  uint32_t* dst = b.path_pool + at;
  dst[n - 1] = entry_e;
  dst[0] = exit_e;
  x = v0;
  lx = lab(v0, b0.x, combo == 2 ? 0u : 1u);
  for (uint32_t q = n - 2; q >= 1; --q) {
    uint32_t pe = kNone, pu = 0;
    unsigned long long plu = kKeyInf;
    if (!find_pred(g, lab, acc, mode, x, lx, pe, pu, plu)) break;   // found on the first walk
    dst[q] = pe; x = pu; lx = plu;
  }
}

// path of one chosen transition (slot p) with a lane-resident search.  Returns false when
// the search outgrew its label store (caller queues p).
template <class L>
__device__ __forceinline__ bool lane_path(const DevGraph& g, const DevBatch& b, uint64_t p, L& S, int cap) {
  const uint4 pi = b.pair_info[p];
  const int mode = (int)(pi.z >> 16);
  const uint32_t bound = pi.x;
  const uint32_t i = (uint32_t)b.choice[p - 1], j = (uint32_t)b.choice[p];
  const uint4 a0 = b.cand_desc[((p - 1) * kMaxCand + i) * 2], a1 = b.cand_desc[((p - 1) * kMaxCand + i) * 2 + 1];
  const uint4 b0 = b.cand_desc[(p * kMaxCand + j) * 2], b1 = b.cand_desc[(p * kMaxCand + j) * 2 + 1];
  unsigned long long rk1, rk0;
  lane_search(S, g, g.relax[mode], bound, a0, a1, rk1, rk0, StopAtTarget{a0, b0, b1});
  if (S.ovf) return false;
  int combo = -1;
  const unsigned long long key = route_key(StoreLabel<L>{S}, a0, b0, b1, &combo);
  path_walk(g, b, p, SearchPathLabels<L>{S}, mode, a0, a1, b0, b1, rk1, rk0, key, combo, cap);
  return true;
}

// path_walk for the ball tier: canonical predecessors from the rows (ball_pred_step), one
// probe pair per walked node instead of one per examined in-edge
// (r1_0 / r0_0: both exits' rows of the target road, already probed for the route key)
__device__ void path_walk_ball(const DevGraph& g, const DevBatch& b, uint64_t p, const BallPathLabels& lab, int mode,
                               const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1,
                               unsigned long long key, int combo, int cap, const uint4& r1_0, const uint4& r0_0) {
  const uint32_t acc = mode_access(mode);
  const uint32_t n1a = a1.y, n0a = a1.x;
  const unsigned long long rk1 = lab.rk1, rk0 = lab.rk0;
  uint32_t* inl = b.path_inline + p * kInlinePath;
  if (combo <= 1) {
    b.route_dist[p] = key_dist(key);
    b.path_sab[p] = make_uint2(a0.y, b0.y);
    inl[0] = combo == 0 ? g.road_fwd[a0.x] : g.road_rev[a0.x];
    b.path_cnt[p] = 1;
    b.path_off[p] = 0;
    return;
  }
  const uint32_t entry_e = combo == 2 ? g.road_fwd[b0.x] : g.road_rev[b0.x];
  const uint32_t v0 = combo == 2 ? b1.x : b1.y, side0 = combo == 2 ? 0u : 1u;
  auto label_at = [&](const uint4& r1, const uint4& r0, uint32_t side) {
    return side ? ball_label(rk1, row_key1(r1), rk0, row_key1(r0)) : ball_label(rk1, row_key0(r1), rk0, row_key0(r0));
  };
  const unsigned long long lx0 = label_at(r1_0, r0_0, side0);
  // first walk: edges shifted into registers (front = travel order), stored after the walk
  uint32_t n = 1, x = v0, side = side0;
  unsigned long long lx = lx0;
  uint4 r1 = r1_0, r0 = r0_0;
  uint32_t pr[kInlinePath];
#pragma unroll
  for (int q = 0; q < kInlinePath; ++q) pr[q] = entry_e;
  for (int guard = 0;; ++guard) {
    if (lx == kKeyInf || guard > cap) { trace_fail(b, p, kErrRounds); return; }
    if ((x == n1a && lx == rk1) || (x == n0a && lx == rk0)) break;
    uint4 rec;
    unsigned long long plu;
    if (!ball_pred_step(g, lab, acc, mode, x, lx, r1, r0, side, rec, plu)) { trace_fail(b, p, kErrRounds); return; }
#pragma unroll
    for (int q = kInlinePath - 1; q > 0; --q) pr[q] = pr[q - 1];
    pr[0] = rec.x;
    ++n;
    x = rec.y;
    side = rec.z & 1u;   // the edge's start: node0 of its road when it runs forward
    lab.rows(rec.z >> 1, r1, r0);
    lx = label_at(r1, r0, side);
  }
  const uint32_t exit_e = (x == n1a) ? g.road_fwd[a0.x] : g.road_rev[a0.x];
#pragma unroll
  for (int q = kInlinePath - 1; q > 0; --q) pr[q] = pr[q - 1];
  pr[0] = exit_e;
  ++n;
  b.route_dist[p] = key_dist(key);
  b.path_sab[p] = make_uint2(a0.y, b0.y);
  b.path_cnt[p] = n;
  if (n <= (uint32_t)kInlinePath) {
#pragma unroll
    for (int q = 0; q < kInlinePath; ++q)
      if ((uint32_t)q < n) inl[q] = pr[q];
    b.path_off[p] = 0;
    return;
  }
  // long path: pool slot, second walk writing in travel order
  const uint32_t at = atomicAdd(&b.ctl[0], n);
  if ((uint64_t)at + n > b.path_cap) { atomicOr(&b.ctl[2], kErrPathOverflow); b.path_off[p] = kNone; return; }
  b.path_off[p] = at;
  uint32_t* dst = b.path_pool + at;
  dst[n - 1] = entry_e;
  dst[0] = exit_e;
  x = v0; side = side0; r1 = r1_0; r0 = r0_0; lx = lx0;
  for (uint32_t q = n - 2; q >= 1; --q) {
    uint4 rec;
    unsigned long long plu;
    if (!ball_pred_step(g, lab, acc, mode, x, lx, r1, r0, side, rec, plu)) break;   // found on the first walk
    dst[q] = rec.x;
    x = rec.y;
    side = rec.z & 1u;
    lab.rows(rec.z >> 1, r1, r0);
    lx = label_at(r1, r0, side);
  }
}

// path ball tier: one lane per chosen transition whose bound fits the ball radius; the
// others go to the search tiers (rl_routes_0 reused after K2, count ctl[8])
#ifndef RM_PATHS_WPE
#define RM_PATHS_WPE 1
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RM_PATHS_WPE))) k_paths_ball(DevGraph g, DevBatch b) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b.perm_paths) {   // locality order: the pair whose source state is the r-th sorted state
    const uint64_t r = (uint64_t)xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    if (r >= b.P) return;
    p = (uint64_t)b.perm_paths[r] + 1u;
  }
  if (p >= b.P) return;
  // the slot's loads issued together (every slot < P holds a choice and a chain flag), the
  // filters after them
  const uint32_t k = b.slot_trace[p];
  const int8_t cj = b.choice[p], ci = b.choice[p ? p - 1 : 0];
  const uint8_t cs = b.chain_start[p];
  const uint32_t o = b.trace_off[k], S = b.n_states[k];
  const uint32_t s = (uint32_t)(p - o);
  if (s < 1 || s >= S || cs || cj < 0) return;
  const uint4 pi = b.pair_info[p];
  const int mode = (int)(pi.z >> 16);
  const uint32_t bound = pi.x;
  const uint32_t i = (uint32_t)ci, j = (uint32_t)cj;
  const uint4 a0 = b.cand_desc[((p - 1) * kMaxCand + i) * 2], a1 = b.cand_desc[((p - 1) * kMaxCand + i) * 2 + 1];
  const uint4 b0 = b.cand_desc[(p * kMaxCand + j) * 2], b1 = b.cand_desc[(p * kMaxCand + j) * 2 + 1];
  unsigned long long rk1, rk0;
  exit_keys(a0, bound, rk1, rk0);
  const bool fits = (g.ball_mask >> mode) & 1u;   // beyond the radius: when the route is exact (ball_exact_limit)
  uint2 h1 = make_uint2(0u, 1u), h0 = h1;
  if (fits) {   // both headers loaded together
    const uint2* hp = g.ball_hdr[mode];
    const uint2 x1 = hp[a1.y], x0 = hp[a1.x];
    if (rk1 != kKeyInf) h1 = x1;
    if (rk0 != kKeyInf) h0 = x0;
  }
  if (!fits || h1.y == 0u || h0.y == 0u) {
    b.rl_routes_0[atomicAdd(&b.ctl[8], 1u)] = (uint32_t)p;
    return;
  }
  const BallPathLabels lab{g.ball_ent[mode], h1, h0, rk1, rk0, g.ball_road_mask};
  // the target road's rows once for both entry labels (and the walk's first node)
  uint4 r1 = make_uint4(kNone, kBallNoDist, kBallNoDist, 0u), r0 = r1;
  if (d_spf(b0) || d_spr(b0)) lab.rows(b0.x, r1, r0);
  const unsigned long long lab0 = d_spf(b0) ? ball_label(rk1, row_key0(r1), rk0, row_key0(r0)) : kKeyInf;
  const unsigned long long lab1 = d_spr(b0) ? ball_label(rk1, row_key1(r1), rk0, row_key1(r0)) : kKeyInf;
  int combo = -1;
  const unsigned long long key = route_key_vals(a0, b0, b1, lab0, lab1, &combo);
  const uint32_t lim = ball_exact_limit(bound, g.ball_radius[mode], rk1, rk0);
  if (lim != kNone && (key == kKeyInf || key_dist(key) > lim)) {   // not decided by the tables
    b.rl_routes_0[atomicAdd(&b.ctl[8], 1u)] = (uint32_t)p;
    return;
  }
  path_walk_ball(g, b, p, lab, mode, a0, a1, b0, b1, key, combo, (int)kBallMaxKeys, r1, r0);
}

// path lane tier: one lane per chosen transition, labels in registers.  With `listed`,
// thread q takes the q-th transition the ball tier handed over.
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RM_LANE_WPE))) k_paths_lane(DevGraph g, DevBatch b, int listed) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  const uint64_t q0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t p = q0;
  if (listed) {   // grid-stride over the ball tier's hand-overs
    const uint32_t n = b.ctl[8];
    for (uint64_t q = q0; q < n; q += (uint64_t)gridDim.x * blockDim.x) {
      RegLabels S;
      if (!lane_path(g, b, b.rl_routes_0[q], S, kLaneCap)) b.rl_paths_a[atomicAdd(&b.ctl[4], 1u)] = b.rl_routes_0[q];
    }
    return;
  } else {
    if (b.perm_paths) {
      const uint64_t r = (uint64_t)xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
      if (r >= b.P) return;
      p = (uint64_t)b.perm_paths[r] + 1u;
    }
    if (p >= b.P) return;
    const uint32_t k = b.slot_trace[p];
    const uint32_t o = b.trace_off[k];
    const uint32_t s = (uint32_t)(p - o);
    if (s < 1 || s >= b.n_states[k]) return;
    if (b.chain_start[p] || b.choice[p] < 0) return;
  }
  RegLabels S;
  if (!lane_path(g, b, p, S, kLaneCap)) {
    const uint32_t q = atomicAdd(&b.ctl[4], 1u);
    b.rl_paths_a[q] = (uint32_t)p;
  }
}

// path second register tier
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) k_paths_reg2(DevGraph g, DevBatch b) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  const uint32_t n_items = b.ctl[4];
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n_items; q += gridDim.x * blockDim.x) {
    const uint32_t p = b.rl_paths_a[q];
    RegLabelsT<kTier2Cap> S;
    if (!lane_path(g, b, p, S, kTier2Cap)) {
      const uint32_t x = atomicAdd(&b.ctl[6], 1u);
      b.rl_paths_b[x] = p;
    }
  }
}

// ------------------------------------------------------------------------------------------
// K2 wave tier: one wave per (pair, source) item that outgrew both lane tiers; the
// source is searched alone in a hash of H (source, node) labels.  Returns false when the
// search outgrew the hash (the caller hands the item to the next tier).
template <int H, int W = kWave>
__device__ bool routes_search_item(SearchSmem<H, false>& sm, uint4* s_src, const DevGraph& g, const DevBatch& b,
                                   uint32_t t) {
  const int lane = grp_lane<W>();
  const uint64_t p = b.src_item[t];
  const uint4 pi = b.pair_info[p];
  const uint32_t i = t - b.src_off[p];
  const uint32_t KB = (pi.z >> 8) & 0xffu;
  const int mode = (int)(pi.z >> 16);
  const uint32_t bound = pi.x, tmax = pi.y;
  const uint32_t base = b.trans_off[p];
  if (lane < 2) s_src[lane] = b.cand_desc[((p - 1) * kMaxCand + i) * 2 + lane];
  grp_sync<W>();
  bounded_search<H, false, W>(sm, g, mode, bound, s_src, 1, 0u,
                              SearchTargets{b.cand_desc + p * kMaxCand * 2, KB, b.search_delta});
  const bool ok = !sm.ovf;
  if (ok) {
    const bool turn = b.route_d != nullptr;   // the batch has turn costs: every route's distance term
    unsigned long long rk1 = kKeyInf, rk0 = kKeyInf;
    double gcp = 0.0;
    if (turn) { exit_keys(s_src[0], bound, rk1, rk0); gcp = b.gc[p]; }
    for (uint32_t j = lane; j < KB; j += W) {
      const uint4 t0 = b.cand_desc[(p * kMaxCand + j) * 2], t1 = b.cand_desc[(p * kMaxCand + j) * 2 + 1];
      int combo = -1;
      const unsigned long long key = route_key(HashLabel<H, false>{sm, 0u}, s_src[0], t0, t1, &combo);
      uint32_t out = kRouteInvalid;
      if (key != kKeyInf && key_dist(key) <= bound && key_time(key) <= tmax) out = key_dist(key);
      b.route[base + i * KB + j] = out;
      if (turn) {   // the route's turn weight (rule 3b) from the same labels
        bool wok = true;
        const uint32_t u = (out == kRouteInvalid || !pi.w)
                               ? 0u
                               : search_turn_walk(g, HashPathLabel<H, false>{sm}, mode, s_src[0], s_src[1], t0, t1, rk1, rk0,
                                                  combo, wok);
        if (!wok) trace_fail(b, p, kErrRounds);
        b.route_d[base + i * KB + j] = route_term(out, u, pi.w, gcp);
      }
    }
  }
  grp_sync<W>();
  return ok;
}

// LDS tiers (round 4).  With early termination most searches end a few blocks past their targets
// and touch tens of nodes: the group tier runs four of them per wave, 16 lanes and a kGrpH-slot
// hash each (four searches in the LDS of one); what outgrows it goes to the 512-slot wave tier
// (10 KB, 16 waves per CU), then to the 4096-slot one (80 KB, 2 waves per CU).  Hand-over lists:
// group tier <- rl_routes_b (ctl[5]) -> rl_routes_a (ctl[11], free once tier 2 has run) -> 512
// tier -> rl_routes_0 (ctl[13], free once the lane tier has run) -> 4096 tier -> rl_routes_c.
#ifndef RM_GRP_H
#define RM_GRP_H 256
#endif
#ifndef RM_GRP_PATH_H
#define RM_GRP_PATH_H 128   // path searches are single-target: smaller (C3 radius 0: 10.3 -> 7.4 ms at 128)
#endif
constexpr int kGrpH = RM_GRP_H;
constexpr int kGrpPathH = RM_GRP_PATH_H;
constexpr int kGrpW = 16;
constexpr uint32_t kGrpGrid = 4096;   // blocks of the group tiers (grid-stride over their lists)
// short: a small run's short hand-over chain (Matcher::run_small, round 6): the group tier takes
// the ball tier's hand-overs (rl_routes_0, ctl[1]) itself and the 4096-slot tier takes the group
// tier's; the lane, second register and 512-slot tiers are not launched (three launches fewer;
// every tier is exact, so the routes are the same)
__global__ void __launch_bounds__(64) k_routes_grp(DevGraph g, DevBatch b, int short_chain) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  __shared__ SearchSmem<kGrpH, false> sm[kWave / kGrpW];
  __shared__ uint4 s_src[kWave / kGrpW][2];
  const int gi = threadIdx.x / kGrpW;
  const uint32_t n_items = short_chain ? b.ctl[1] : b.ctl[5];
  const uint32_t* list = short_chain ? b.rl_routes_0 : b.rl_routes_b;
  for (uint32_t item = blockIdx.x * (kWave / kGrpW) + gi; item < n_items; item += gridDim.x * (kWave / kGrpW)) {
    const uint32_t t = list[item];
    if (!routes_search_item<kGrpH, kGrpW>(sm[gi], s_src[gi], g, b, t) && grp_lane<kGrpW>() == 0)
      b.rl_routes_a[atomicAdd(&b.ctl[11], 1u)] = t;
  }
}

__global__ void __launch_bounds__(64) k_routes_wave_s(DevGraph g, DevBatch b) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  __shared__ SearchSmem<kMidH, false> sm;
  __shared__ uint4 s_src[2];
  const uint32_t n_items = b.ctl[11];
  for (uint32_t item = blockIdx.x; item < n_items; item += gridDim.x) {
    const uint32_t t = b.rl_routes_a[item];
    if (!routes_search_item<kMidH>(sm, s_src, g, b, t) && threadIdx.x == 0) b.rl_routes_0[atomicAdd(&b.ctl[13], 1u)] = t;
  }
}

__global__ void __launch_bounds__(64) k_routes_wave(DevGraph g, DevBatch b, int short_chain) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  __shared__ SearchSmem<kBigH, false> sm;
  __shared__ uint4 s_src[2];
  const uint32_t n_items = short_chain ? b.ctl[11] : b.ctl[13];   // (short: the group tier's hand-overs)
  const uint32_t* list = short_chain ? b.rl_routes_a : b.rl_routes_0;
  for (uint32_t item = blockIdx.x; item < n_items; item += gridDim.x) {
    const uint32_t t = list[item];
    if (!routes_search_item<kBigH>(sm, s_src, g, b, t) && threadIdx.x == 0) b.rl_routes_c[atomicAdd(&b.ctl[9], 1u)] = t;
  }
}

// Global-memory tier (routes and paths): searches that outgrew the 4096-slot LDS hash (route
// bounds of many kilometres: sparse sampling with a large breakage_distance) run here with a
// kGlobalH-slot hash in a per-block global scratch.  What outgrows even this fails ITS trace
// only (trace_err), never the batch.
constexpr int kGlobalH = 1 << 17;
constexpr int kGlobalGrid = 32;
using GlobalRouteSmem = SearchSmem<kGlobalH, false>;
using GlobalPathSmem = SearchSmem<kGlobalH, true>;

__global__ void __launch_bounds__(64) k_routes_global(DevGraph g, DevBatch b, GlobalPathSmem* scratch) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  __shared__ uint4 s_src[2];
  GlobalRouteSmem& sm = *reinterpret_cast<GlobalRouteSmem*>(scratch + blockIdx.x);
  const uint32_t n_items = b.ctl[9];
  for (uint32_t item = blockIdx.x; item < n_items; item += gridDim.x) {
    const uint32_t t = b.rl_routes_c[item];
    if (!routes_search_item<kGlobalH>(sm, s_src, g, b, t) && threadIdx.x == 0) trace_fail(b, b.src_item[t], kErrSearchOverflow);
  }
}

// ------------------------------------------------------------------------------------------
// K3 k_viterbi: 16 lanes per trace, 4 traces per wave; lane j owns candidate j of the
// current layer.  A wave64 VALU instruction costs a SIMD four cycles, so the layer
// recurrence is packed four traces to an instruction (one trace per wave would spend
// ~4x the issue slots on the same work), and the recurrence is issue-bound, so the layer
// body is cut to the fewest instructions: a group is a DPP row, the previous layer's costs
// stay in registers (lane i holds cost i) and reach every lane of the row by row_newbcast
// moves (no LDS round trip, no barrier), and routes are staged as fp64 metres (+inf when
// invalid) so a source costs three fp64 operations and a compare.  Each group streams its trace through LDS in
// chunks of <= 16 layers / <= kVitRoutes routes: one lane describes one layer, a 16-lane
// scan lays the chunk out, and routes / emission rows arrive with coalesced loads a chunk
// ahead (below, "the chunk pipeline").  No global store is issued inside a chunk (gfx9
// loads and stores share vmcnt): back-pointer rows are buffered in LDS and flushed, with
// the chunk's chain-start flags, once per chunk.
constexpr int kVitChunk = 16;     // layers per staged chunk (one per lane of the group)
#ifndef RM_VIT_WPE
#define RM_VIT_WPE 3   // 2,500 C2 waves over 1,024 SIMDs must be resident at once (also LDS: VitGroup)
#endif
#ifndef RM_VIT_ROUTES
#define RM_VIT_ROUTES 256
#endif
constexpr int kVitRoutes = RM_VIT_ROUTES;  // routes per staged chunk and group
constexpr int kVitBt = 64;        // layers per backtrace staging block
struct VitGroup {
  // LDS per wave bounds K3's residency (C2: 2,500 waves over 256 CUs need <= 14.5 KB per
  // wave for one round), so the backtrace staging aliases the chunk's routes; a backtrace
  // inside a chunk re-stages them from HBM afterwards (chain breaks are rare)
  union {
    double route_m[kVitRoutes];   // route length in metres ((double)cm * 0.01), +inf when invalid
    uint4 bst[kVitBt];            // backtrace staging
  };
  float sq[kVitChunk][16];
  double gc[kVitChunk];
  uint32_t kb[kVitChunk], rel[kVitChunk];
  uint4 bpo[kVitChunk + 1];       // this chunk's back-pointer rows (16 x u8); + a spare row
  uint8_t cs[kVitChunk + 1];      // this chunk's chain-start flags (+ spare)
  uint8_t ch[kVitBt];             // choices of one backtrace block
  uint32_t nch, done, w, pad;
#if defined(RM_VIT_PAD) && RM_VIT_PAD > 0
  uint32_t padv[RM_VIT_PAD];      // A/B of the four groups' LDS bank alignment
#endif
};

static_assert(sizeof(VitGroup) >= (kVitRoutes + 15 + 7 * 16 + 1) * sizeof(double), "K3 prefetch reads (8 source rows) stay inside VitGroup");

// lane I of this lane's 16-lane row (DPP row_newbcast; rows are the K3 groups)
template <int I>
__device__ __forceinline__ double row_bcast(double v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + I, 0xf, 0xf, false);   // one v_mov_b64_dpp
}

// best / arg over sources I.. prevK-1 of this lane's target: cost of source i (lane i's cj)
// plus |route_m - gc| / beta, the first strict minimum in source order.
// Sources go in blocks of four under a group-uniform guard (every lane of the row is active
// inside it): the block's four LDS loads issue together and complete under one wait, then
// each source costs a subtract, a fused multiply-add, a compare, a min and one select.  Sources past
// prevK in the last block need no guard: lanes i >= prevK hold cj = +inf (every layer sets
// cost +inf past its KB), and +inf (or NaN from the unstaged LDS they read) never wins.
template <int I, bool TURN>
__device__ __forceinline__ void vit_src(double& best, int& arg, double cj, double rm, double gcl, double inv_beta) {
  // fma(|route_m - gc|, 1/beta, cost of source i): one rounding, as the oracle's fma; an
  // invalid route is +inf and stays +inf.  With turn costs (rule 3b) the staged value is the
  // distance term turn_m + |route_m - gc| itself (route_d, formed by K2 as the oracle forms it).
  const double d = TURN ? rm : fabs(rm - gcl);
  const double c = __builtin_fma(d, inv_beta, row_bcast<I>(cj));
  const bool take = c < best;
  best = __builtin_fmin(best, c);   // = c exactly when take (no NaN reaches here, costs >= 0)
  arg = take ? I : arg;
}
template <int B, bool TURN>
__device__ __forceinline__ void vit_min(double& best, int& arg, double cj, const double* dp, uint32_t KB,
                                        uint32_t prevK, double gcl, double inv_beta, const double* rm0) {
  if constexpr (B < 4) {
    if ((uint32_t)(4 * B) < prevK) {
      double rm[4];
      if constexpr (B == 0) {   // block 0 was loaded at the end of the previous layer
#pragma unroll
        for (int x = 0; x < 4; ++x) rm[x] = rm0[x];
      } else {
#pragma unroll
        for (int x = 0; x < 4; ++x) rm[x] = dp[(4 * B + x) * KB];   // past prevK: never selected
#pragma unroll
        for (int x = 0; x < 4; ++x) __asm__ volatile("" : "+v"(rm[x]));   // keep the loads together
      }
      vit_src<4 * B + 0, TURN>(best, arg, cj, rm[0], gcl, inv_beta);
      vit_src<4 * B + 1, TURN>(best, arg, cj, rm[1], gcl, inv_beta);
      vit_src<4 * B + 2, TURN>(best, arg, cj, rm[2], gcl, inv_beta);
      vit_src<4 * B + 3, TURN>(best, arg, cj, rm[3], gcl, inv_beta);
      vit_min<B + 1, TURN>(best, arg, cj, dp, KB, prevK, gcl, inv_beta, rm0);
    }
  }
}


__device__ __forceinline__ double shfl_xor_d(double v, int m, int width) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __shfl_xor((int)(uint32_t)u, m, width), hi = __shfl_xor((int)(uint32_t)(u >> 32), m, width);
  return __longlong_as_double(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo);
}

// back-pointer rows and chain-start flags of chunk layers [0, n) to HBM (layer l at slot l0 + l;
// csm: the chunk's chain-start flags as a wave mask, bit `lane` = layer j of lane j's group)
__device__ __forceinline__ void vit_flush_m(const DevBatch& b, const VitGroup& gs, uint64_t l0, uint32_t n, int j,
                                            unsigned long long csm) {
  if ((uint32_t)j < n) {
    *reinterpret_cast<uint4*>(b.bp + (l0 + j) * kMaxCand) = gs.bpo[j];
    b.chain_start[l0 + j] = __builtin_amdgcn_inverse_ballot_w64(csm) ? 1 : 0;
  }
}

// Backtrace of the chain ending at layer `end` (lane j holds cost j of that layer, K
// candidates).  Winner = lowest cost, ties to the lowest j.  Rows are staged 64 layers
// per block (four coalesced loads per lane); lane 0 of the group walks them in LDS and
// the block's choices leave as one store per lane.
__device__ void backtrace_chain(const DevBatch& b, VitGroup& gs, uint32_t o, uint32_t end, uint32_t K, int j, double cj) {
  double bc = (j < (int)K) ? cj : __longlong_as_double(0x7ff0000000000000ll);
  int bj = (j < (int)K) ? j : 1 << 20;
  for (int m = 1; m < 16; m <<= 1) {
    const double oc = shfl_xor_d(bc, m, 16);
    const int oj = __shfl_xor(bj, m, 16);
    if (oc < bc || (oc == bc && oj < bj)) { bc = oc; bj = oj; }
  }
  uint32_t w = (uint32_t)bj;
  __threadfence_block();  // this wave's bp stores are visible to its loads
  int t = (int)end;
  for (;;) {
    uint4 row[kVitBt / 16];
#pragma unroll
    for (int x = 0; x < kVitBt / 16; ++x) {   // every row load in flight before the LDS stores
      const int lay = t - (j + 16 * x);
      row[x] = make_uint4(0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu);
      if (lay >= 0) row[x] = *reinterpret_cast<const uint4*>(b.bp + (uint64_t)(o + lay) * kMaxCand);
    }
#pragma unroll
    for (int x = 0; x < kVitBt / 16; ++x) gs.bst[j + 16 * x] = row[x];
    wave_sync();
    if (j == 0) {
      uint32_t l = 0, done = 0;
      for (; l < (uint32_t)kVitBt && t - (int)l >= 0;) {
        gs.ch[l] = (uint8_t)w;
        const uint32_t nb = reinterpret_cast<const uint8_t*>(&gs.bst[l])[w];
        ++l;
        if (nb == 255u) { done = 1; break; }
        w = nb;
      }
      if (t - (int)l < 0) done = 1;
      gs.nch = l; gs.done = done; gs.w = w;
    }
    wave_sync();
    const uint32_t n = gs.nch;
#pragma unroll
    for (int x = 0; x < kVitBt / 16; ++x)
      if ((uint32_t)(j + 16 * x) < n) b.choice[o + t - (j + 16 * x)] = (int8_t)gs.ch[j + 16 * x];
    const bool done = gs.done != 0;
    w = gs.w;
    t -= (int)n;
    wave_sync();
    if (done) break;
  }
}

struct VitLayerDesc {
  uint32_t kb, cnt, off;
  double gc;
};

// the loads behind a VitLayerDesc, kept raw: k_viterbi_w loads them a chunk ahead and forms the
// description (vit_cook) only when it lays that chunk out, so nothing waits on them early
struct VitLayerRaw {
  uint32_t kb, ka, off;
  double gc;
};
__device__ __forceinline__ VitLayerRaw vit_raw(const DevBatch& b, uint32_t o, uint32_t S, uint32_t s0, int j) {
  const uint64_t lq = o + min(s0 + (uint32_t)j, S - 1);
  const uint64_t lp = lq == o ? o : lq - 1;
  VitLayerRaw r;
  r.kb = b.cand_n[lq];
  r.ka = b.cand_n[lp];
  r.off = b.trans_off[lq];
  r.gc = b.gc[lq];
  return r;
}
__device__ __forceinline__ VitLayerDesc vit_cook(const VitLayerRaw& r, uint32_t S, uint32_t s0, int j) {
  const uint32_t sl = s0 + j;
  const bool vq = sl < S;
  VitLayerDesc d;
  d.off = r.off;
  d.kb = vq ? r.kb : 0u;
  d.cnt = (vq && sl >= 1) ? r.ka * d.kb : 0u;
  d.gc = (vq && sl >= 1) ? r.gc : 0.0;
  return d;
}

// layer s0 + j of a trace: candidate count, route count, route offset, gc
__device__ __forceinline__ VitLayerDesc vit_describe(const DevBatch& b, uint32_t o, uint32_t S, uint32_t s0, int j) {
  const uint32_t sl = s0 + j;
  const bool vq = sl < S;
  const uint64_t lq = o + min(sl, S - 1);
  const uint64_t lp = lq == o ? o : lq - 1;
  const uint32_t kb_raw = b.cand_n[lq], ka_raw = b.cand_n[lp];
  const double g_raw = b.gc[lq];
  VitLayerDesc d;
  d.off = b.trans_off[lq];
  d.kb = vq ? kb_raw : 0u;
  d.cnt = (vq && sl >= 1) ? ka_raw * d.kb : 0u;
  d.gc = (vq && sl >= 1) ? g_raw : 0.0;
  return d;
}

// ------------------------------------------------------------------------------------------
// K3 (round 2, v3): one wave per trace, one lane per transition.  A layer's K_A x K_B
// transitions are spread over the wave as lane = (target j, source i) with W = 4, 8 or 16
// source lanes per target (the smallest power of two >= K_A; 64/W targets per pass, one pass
// for K_A <= 4 or K_A, K_B <= 8): every transition costs one fused multiply-add at once, the
// minimum over sources is a DPP butterfly inside the W lanes (quad_perm, row_half_mirror,
// row_mirror) and the arg-min a ballot of "c == min" (first set bit = lowest i, the strict-<
// scan's tie rule).  10,000 C2 traces are 10,000 independent waves (8 per SIMD resident), so
// the per-layer latency chain (LDS read -> fma -> butterfly -> ballot -> LDS write) of one
// trace hides behind the others; all control flow is wave-uniform (scalar branches).
// Routes reach LDS per chunk of <= 16 layers / kV3Routes routes as fp64 metres (+inf when
// invalid, an +inf sentinel for idle lanes); the next chunk's routes and emission rows are
// loaded into registers while this chunk runs, and the chunk after that is described then.
// Measured on C2 (bit-exact): 1.01 ms against 0.75 ms for k_viterbi.  Per trace-layer it issues
// 65 VALU + 70 SALU + 10 LDS instructions against 48 + 22 + 5 (C2's typical layer has K = 4,
// so 16 of 64 lanes work either way, and the wave-uniform control is paid per trace instead of
// per four), and 10,000 waves need two rounds of 8 per SIMD (8,000 traces: 0.75 ms).  Round 4:
// it runs the small batches (launch_viterbi below), where its shorter layer chain wins.
#ifndef RM_VIT3_WPE
#define RM_VIT3_WPE 4   // it runs batches of <= 4,096 traces: <= 4 waves per SIMD; 128 VGPRs hold the prefetch
#endif
constexpr int kV3Routes = 384;               // routes per staged chunk
constexpr int kV3Chunk = 16;                 // layers per staged chunk (one per lane 0..15)
constexpr int kV3Regs = kV3Routes / kWave;   // route registers per lane for the next chunk
struct Vit3Smem {
  union {
    double route_m[kV3Routes + 2];           // [kV3Routes] = +inf: the route of an idle lane
    struct {
      uint4 bst[kWave];                      // backtrace staging (64 back-pointer rows)
      uint8_t ch[kWave];
    } bt;
  };
  float sq[kV3Chunk][kMaxCand];
  double cost[2][kMaxCand];                  // previous / next layer costs (ping-pong)
  uint4 bpo[kV3Chunk];                       // this chunk's back-pointer rows
  uint32_t nch, done, w, pad;
};
static_assert(sizeof(Vit3Smem) <= 5120, "K3 v3 must keep 8 waves per SIMD (32 per CU) within LDS");

struct V3Chunk {
  uint32_t s0, C, nroutes, rbase;
  uint32_t kbrel;   // lane t < C: K_B of layer s0 + t | offset of its routes in the chunk << 8
  double gc;        // lane t < C: gc of layer s0 + t
};

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo);
}

// minimum over each aligned group of W lanes, in every lane of the group (all lanes active)
template <int W>
__device__ __forceinline__ double group_min(double c) {
  c = __builtin_fmin(c, dpp_d<0xB1>(c));                      // quad_perm [1,0,3,2]
  c = __builtin_fmin(c, dpp_d<0x4E>(c));                      // quad_perm [2,3,0,1]
  if constexpr (W >= 8) c = __builtin_fmin(c, dpp_d<0x141>(c));   // row_half_mirror (x <-> 7-x)
  if constexpr (W >= 16) c = __builtin_fmin(c, dpp_d<0x140>(c));  // row_mirror (x <-> 15-x)
  return c;
}

__device__ __forceinline__ double readlane_d(double v, uint32_t l) {
  const unsigned long long u = __double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, (int)l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), (int)l);
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// chunk from s0: lanes 0..15 describe layers s0..s0+15 (d); the leading layers whose routes
// fit kV3Routes form the chunk (at least one: a layer holds <= 256 routes)
__device__ __forceinline__ V3Chunk v3_layout(const VitLayerDesc& d, uint32_t s0, uint32_t S, int lane) {
  const int j = lane & 15;
  uint32_t incl = d.cnt;
#pragma unroll
  for (int x = 1; x < 16; x <<= 1) {
    const uint32_t u = __shfl_up(incl, x, 16);
    if (j >= x) incl += u;
  }
  const uint32_t fit = (uint32_t)(__ballot(lane < 16 && s0 + (uint32_t)lane < S && incl <= (uint32_t)kV3Routes) & 0xffffull);
  V3Chunk c;
  c.s0 = s0;
  // wave-uniform values live in SGPRs (the layer loop and its branches are scalar)
  c.C = (uint32_t)__builtin_amdgcn_readfirstlane((int)__builtin_ctz(~fit | 0x10000u));
  c.nroutes = c.C ? (uint32_t)__builtin_amdgcn_readlane((int)incl, (int)c.C - 1) : 0u;   // C 0: past the trace
  c.rbase = (uint32_t)__builtin_amdgcn_readfirstlane((int)d.off);
  c.kbrel = d.kb | ((incl - d.cnt) << 8);
  c.gc = d.gc;
  return c;
}

// The next chunk's routes (or, with turn costs, its distance terms) and emission rows, loaded
// into registers one chunk ahead.  Every load is unconditional, at a clamped address inside the
// batch (a chunk past the trace's end reads its last layer again; staging ignores lanes past
// nroutes): a conditional load leaves a register merge behind it, and the copy that merge
// needs makes the wave wait for the load at once -- measured, each chunk then paid the full
// memory latency before its first layer (C1's 1,000-layer trace: 0.52 ms in K3).
// (the emission row as a native vector: HIP's float4 is a union-backed class, which the
// compiler kept in scratch across the chunk loop -- one more wait per chunk)
typedef float v3_f4 __attribute__((ext_vector_type(4)));
template <bool TURN>
struct V3Regs {
  uint32_t rv[TURN ? 1 : kV3Regs];
  double rd[TURN ? kV3Regs : 1];
  v3_f4 sv;
};

template <bool TURN>
__device__ __forceinline__ void v3_load(const DevBatch& b, uint32_t o, uint32_t S, const V3Chunk& c, int lane,
                                        V3Regs<TURN>& r) {
  const uint32_t rlast = c.nroutes ? c.nroutes - 1u : 0u;
#pragma unroll
  for (int x = 0; x < kV3Regs; ++x) {
    const uint32_t q = c.rbase + min((uint32_t)(lane + kWave * x), rlast);
    if constexpr (TURN) r.rd[x] = b.route_d[q];
    else r.rv[x] = b.route[q];
  }
  const uint32_t s0 = min(c.s0, S - 1u);
  const uint32_t C = max(min(c.C, S - s0), 1u);
  const v3_f4* src = reinterpret_cast<const v3_f4*>(b.cand_sq) + (uint64_t)(o + s0) * (kMaxCand / 4);
  r.sv = src[min((uint32_t)lane, C * (kMaxCand / 4) - 1u)];
}

template <bool TURN>
__device__ __forceinline__ void v3_stage_routes(Vit3Smem& sm, const V3Chunk& c, int lane, const V3Regs<TURN>& r) {
  const double INF = __longlong_as_double(0x7ff0000000000000ll);
#pragma unroll
  for (int x = 0; x < kV3Regs; ++x)
    if ((uint32_t)(lane + kWave * x) < c.nroutes) {
      // with turn costs (rule 3b) the staged value is the distance term route_d (turn_m +
      // |route_m - gc|, +inf when invalid) in place of the route's metres
      if constexpr (TURN) sm.route_m[lane + kWave * x] = r.rd[x];
      else sm.route_m[lane + kWave * x] = r.rv[x] == kRouteInvalid ? INF : (double)r.rv[x] * 0.01;
    }
}

// back-pointer rows / chain flags (csm: bit l = layer l starts a chain) of chunk layers [0, n) to HBM
__device__ __forceinline__ void v3_flush(const DevBatch& b, const Vit3Smem& sm, uint64_t l0, uint32_t n, int lane,
                                         uint32_t csm) {
  if ((uint32_t)lane < n) {
    *reinterpret_cast<uint4*>(b.bp + (l0 + lane) * kMaxCand) = sm.bpo[lane];
    b.chain_start[l0 + lane] = (uint8_t)((csm >> lane) & 1u);
  }
}

// Backtrace of the chain ending at layer `end` whose costs are sm.cost[cb][0..K): winner =
// lowest cost, ties to the lowest j; rows staged 64 layers at a time, lane 0 walks them.
__device__ void v3_backtrace(const DevBatch& b, Vit3Smem& sm, uint32_t o, uint32_t end, uint32_t K, int cb, int lane) {
  const double INF = __longlong_as_double(0x7ff0000000000000ll);
  const double c = (uint32_t)lane < K ? sm.cost[cb][lane & 15] : INF;
  const double m = group_min<16>(c);
  const uint32_t eq = (uint32_t)(__ballot((uint32_t)lane < K && c == m) & 0xffffull);
  uint32_t w = (uint32_t)__builtin_ctz(eq | 0x10000u);
  __threadfence_block();  // this wave's bp stores are visible to its loads
  int t = (int)end;
  for (;;) {
    const int lay = t - lane;
    uint4 row = make_uint4(0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu);
    if (lay >= 0) row = *reinterpret_cast<const uint4*>(b.bp + (uint64_t)(o + lay) * kMaxCand);
    sm.bt.bst[lane] = row;
    wave_sync();
    if (lane == 0) {
      uint32_t l = 0, done = 0;
      for (; l < (uint32_t)kWave && t - (int)l >= 0;) {
        sm.bt.ch[l] = (uint8_t)w;
        const uint32_t nb = reinterpret_cast<const uint8_t*>(&sm.bt.bst[l])[w];
        ++l;
        if (nb == 255u) { done = 1; break; }
        w = nb;
      }
      if (t - (int)l < 0) done = 1;
      sm.nch = l; sm.done = done; sm.w = w;
    }
    wave_sync();
    const uint32_t n = sm.nch;
    if ((uint32_t)lane < n) b.choice[o + t - lane] = (int8_t)sm.bt.ch[lane];
    const bool done = sm.done != 0;
    w = sm.w;
    t -= (int)n;
    wave_sync();
    if (done) break;
  }
}

// one pass of layer t over targets [j0, j0 + 64/W): lane = (target j0 + lane/W, source lane%W);
// heads (source lane 0) write the target's new cost and back-pointer byte
template <int W, bool TURN>
__device__ __forceinline__ unsigned long long v3_pass(Vit3Smem& sm, int lane, uint32_t j0, uint32_t KB, uint32_t KA,
                                                      uint32_t rel, double gcl, double inv_beta, double inv2s2, int cb,
                                                      uint32_t t, double em4) {
  const double INF = __longlong_as_double(0x7ff0000000000000ll);
  const uint32_t i = (uint32_t)lane & (W - 1), j = j0 + ((uint32_t)lane / W);
  const bool valid = i < KA && j < KB;
  const uint32_t at = valid ? rel + i * KB + j : (uint32_t)kV3Routes;
  const double rm = sm.route_m[at];
  const double ci = sm.cost[cb][i];
  // fma(|route_m - gc|, 1/beta, cost of source i): one rounding, as the oracle; an invalid
  // route, an unreachable source and an idle lane are +inf.  With turn costs (rule 3b) the staged
  // value is the distance term itself.
  const double d = TURN ? rm : fabs(rm - gcl);
  const double c = __builtin_fma(d, inv_beta, ci);
  const double m = group_min<W>(c);
  const unsigned long long eq = __ballot(c == m && m < INF);
  const uint32_t g = (uint32_t)(eq >> ((uint32_t)lane & ~(uint32_t)(W - 1))) & ((1u << W) - 1u);
  const bool head = i == 0u && j < KB;
  // a group has an arg-min exactly when its minimum is finite (some lane equals it); the values
  // are formed in every lane and only the heads store
  const bool fin = m < INF;
  const unsigned long long any = __ballot(head && fin);
  // W = 4 (one pass, j = lane / 4): the emission was read a layer ahead, off this layer's chain
  const double em = W == 4 ? em4 : (double)sm.sq[t][min(j, (uint32_t)kMaxCand - 1u)] * inv2s2;
  const double nc = fin ? m + em : INF;
  const uint8_t bpj = fin ? (uint8_t)__builtin_ctz(g | 0x10000u) : (uint8_t)255;
  if (head) {
    sm.cost[cb ^ 1][j] = nc;
    reinterpret_cast<uint8_t*>(&sm.bpo[t])[j] = bpj;
  }
  return any;
}

template <bool TURN>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RM_VIT3_WPE))) k_viterbi_w(DevBatch b) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  __shared__ Vit3Smem sm;
  const int lane = threadIdx.x;
  const uint32_t k = blockIdx.x;
  const uint32_t o = b.trace_off[k], S = b.n_states[k];
  const MatchOptions op = b.opts[b.trace_opt[k]];
  const double inv2s2 = 1.0 / (2.0 * (double)op.sigma_z * (double)op.sigma_z);
  const double inv_beta = 1.0 / (double)op.beta;
  const double brk = (double)op.breakage_distance;
  const double INF = __longlong_as_double(0x7ff0000000000000ll);
  if (lane < 2 * kMaxCand) (&sm.cost[0][0])[lane] = INF;
  if (lane == 0) sm.route_m[kV3Routes] = INF;
  if (S == 0) return;
  // chunk 0: describe, lay out, load; then describe chunk 1
  V3Chunk cur = v3_layout(vit_describe(b, o, S, 0, lane & 15), 0, S, lane);
  V3Regs<TURN> rg;
  v3_load<TURN>(b, o, S, cur, lane, rg);
  VitLayerRaw dn = vit_raw(b, o, S, cur.C, lane & 15);   // (past S: clamped; vit_cook gives kb 0)
  bool prev_ok = false;
  uint32_t prevK = 0;
  int cb = 0;
  for (;;) {
    v3_stage_routes<TURN>(sm, cur, lane, rg);
    if ((uint32_t)lane < cur.C * (kMaxCand / 4)) reinterpret_cast<v3_f4*>(&sm.sq[0][0])[lane] = rg.sv;
    // the next chunk's routes and emission rows load while this chunk runs (unconditionally:
    // past the trace's end they are never staged)
    const uint32_t s1 = cur.s0 + cur.C;
    const bool has_next = s1 < S;
    const V3Chunk nx = v3_layout(vit_cook(dn, S, s1, lane & 15), s1, S, lane);
    v3_load<TURN>(b, o, S, nx, lane, rg);
    dn = vit_raw(b, o, S, s1 + nx.C, lane & 15);
    // per chunk, once: the back-pointer rows start empty, and which layers' gaps break the chain
    // (layer t of the chunk: bit t); the layers' chain-start flags collect in csm
    if (lane < kV3Chunk) sm.bpo[lane] = make_uint4(0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu);
    const uint32_t brkm = (uint32_t)(__ballot(lane < 16 && (uint32_t)lane < cur.C && cur.s0 + (uint32_t)lane > 0u &&
                                              cur.gc > brk) & 0xffffull);
    uint32_t csm = 0u;
    wave_sync();
    // the emission of target lane / 4 (a W = 4 pass) one layer ahead, off the layer's chain
    double em4n = (double)sm.sq[0][lane >> 2] * inv2s2;
    for (uint32_t t = 0; t < cur.C; ++t) {
      const uint32_t s = cur.s0 + t;
      const uint32_t kr = (uint32_t)__builtin_amdgcn_readlane((int)cur.kbrel, (int)t);
      const uint32_t KB = kr & 0xffu, rel = kr >> 8;
      const double gcl = TURN ? 0.0 : readlane_d(cur.gc, t);   // (with turn costs the staged term holds it)
      const double em4 = em4n;
      bool start = !prev_ok || ((brkm >> t) & 1u) != 0u;
      // the common layer (the chain goes on, K_A <= 4: one W = 4 pass) takes a path of its own
      // past the chain-break, empty-layer and chain-start bookkeeping
      if (KB && !start && prevK <= 4u) {
        const unsigned long long any = v3_pass<4, TURN>(sm, lane, 0u, KB, prevK, rel, gcl, inv_beta, inv2s2, cb, t, em4);
        if (any != 0ull) {
          em4n = (double)sm.sq[min(t + 1u, cur.C - 1u)][lane >> 2] * inv2s2;
          wave_sync();
          prevK = KB;
          cb ^= 1;
          continue;
        }
        start = true;   // no valid transition into this layer: the general path below breaks the chain
      } else if (KB && !start) {   // K_A > 4
        unsigned long long any = 0ull;
        if (prevK <= 8u) {
          any = v3_pass<8, TURN>(sm, lane, 0u, KB, prevK, rel, gcl, inv_beta, inv2s2, cb, t, em4);
          if (KB > 8u) any |= v3_pass<8, TURN>(sm, lane, 8u, KB, prevK, rel, gcl, inv_beta, inv2s2, cb, t, em4);
        } else {
          for (uint32_t j0 = 0; j0 < KB; j0 += 4u)
            any |= v3_pass<16, TURN>(sm, lane, j0, KB, prevK, rel, gcl, inv_beta, inv2s2, cb, t, em4);
        }
        if (any == 0ull) start = true;   // no valid transition into this layer
      }
      em4n = (double)sm.sq[min(t + 1u, cur.C - 1u)][lane >> 2] * inv2s2;
      if (s > 0 && prev_ok && (KB == 0 || start)) {
        // the chain ending at layer s - 1 is complete: its rows [.., s) must be in HBM
        wave_sync();
        v3_flush(b, sm, o + cur.s0, t, lane, csm);
        v3_backtrace(b, sm, o, s - 1, prevK, cb, lane);
        if (t + 1 < cur.C) {   // the backtrace staged through route_m: bring the chunk back
          const double INF = __longlong_as_double(0x7ff0000000000000ll);
          const uint32_t* rp = b.route + cur.rbase;
          const double* dp = b.route_d + cur.rbase;
          __asm__ volatile("" : "+s"(rp), "+s"(dp));   // rare path: keep its addresses out of the loop's registers
#pragma unroll
          for (int x = 0; x < kV3Regs; ++x) {
            const uint32_t q = (uint32_t)(lane + kWave * x);
            if (q < cur.nroutes) {
              if constexpr (TURN) sm.route_m[q] = dp[q];
              else sm.route_m[q] = rp[q] == kRouteInvalid ? INF : (double)rp[q] * 0.01;
            }
          }
        }
      }
      if (KB == 0) {
        csm |= 1u << t;
        prev_ok = false;
        prevK = 0;
        wave_sync();
        continue;
      }
      if (start && lane < kMaxCand)   // a chain starts: cost = emission, back-pointers none
        sm.cost[cb ^ 1][lane] = (uint32_t)lane < KB ? (double)sm.sq[t][lane] * inv2s2 : INF;
      csm |= (start ? 1u : 0u) << t;
      wave_sync();
      prev_ok = true;
      prevK = KB;
      cb ^= 1;
    }
    wave_sync();
    v3_flush(b, sm, o + cur.s0, cur.C, lane, csm);
    wave_sync();
    if (!has_next) break;
    cur = nx;
  }
  if (prev_ok) {
    wave_sync();
    v3_backtrace(b, sm, o, S - 1, prevK, cb, lane);
  }
}

// ------------------------------------------------------------------------------------------
// K3 k_viterbi, the chunk pipeline (round 5).  Round 4's kernel loaded a chunk's routes and
// emission rows at the chunk's start and waited for them there (one HBM round trip per chunk of
// ~10 layers, under 2-3 waves per SIMD), and it guarded each of its 16 route loads and stores by
// its own per-lane branch (~650 instructions per chunk: ~40 % of the kernel's).  Now the next
// chunk is laid out and its routes and emission rows are loaded into registers while this chunk
// runs (the chunk after that is described then), every load is unconditional (vit_load), and
// staging writes every entry (past the chunk: routes / rows never selected -- a source past prevK
// costs +inf, a target past K_B is discarded).  The layer's bookkeeping (chain starts, breaks,
// the backtrace trigger, chain-start flags) is wave masks on the scalar unit.  C2: 0.65 -> 0.51 ms.
template <bool TURN>
struct VitRegs {
  uint32_t rv[TURN ? 1 : kVitRoutes / 16];
  double rd[TURN ? kVitRoutes / 16 : 1];
  v3_f4 sv[4];
};

struct VitChunk {
  uint32_t s0, C, nroutes, rbase;   // group-uniform (C: the smallest over the wave's live groups)
  uint32_t kb, rel;                 // lane j < C: K_B of layer s0 + j, its routes' offset in the chunk
  double gc;
};

// vit_raw for any trace: an empty trace (or a lane past the batch) reads layer 0 of the batch
__device__ __forceinline__ VitLayerRaw vit_raw_any(const DevBatch& b, uint32_t o, uint32_t S, uint32_t s0, int j) {
  const uint64_t lq = S ? o + min(s0 + (uint32_t)j, S - 1) : 0u;
  const uint64_t lp = (S == 0 || lq == o) ? lq : lq - 1;
  VitLayerRaw r;
  r.kb = b.cand_n[lq];
  r.ka = b.cand_n[lp];
  r.off = b.trans_off[lq];
  r.gc = b.gc[lq];
  return r;
}

__device__ __forceinline__ VitChunk vit_layout(const VitLayerDesc& d, uint32_t s0, uint32_t S, int j, int gb) {
  // inclusive scan of the route counts inside the 16-lane row by DPP row_shr adds (bound_ctrl:
  // a lane without a source adds 0), the groups' minimum by readlanes: no LDS round trips
  uint32_t incl = d.cnt;
  incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x111, 0xf, 0xf, true);   // row_shr:1
  incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x112, 0xf, 0xf, true);   // row_shr:2
  incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x114, 0xf, 0xf, true);   // row_shr:4
  incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x118, 0xf, 0xf, true);   // row_shr:8
  const bool live = s0 < S;
  const uint32_t fit = (uint32_t)((__ballot(live && s0 + (uint32_t)j < S && incl <= (uint32_t)kVitRoutes) >> gb) & 0xffffull);
  const uint32_t Cg = live ? (uint32_t)__builtin_ctz(~fit | 0x10000u) : 0x10000u;   // leading layers that fit
  const uint32_t Cw = min(min((uint32_t)__builtin_amdgcn_readlane((int)Cg, 0), (uint32_t)__builtin_amdgcn_readlane((int)Cg, 16)),
                          min((uint32_t)__builtin_amdgcn_readlane((int)Cg, 32), (uint32_t)__builtin_amdgcn_readlane((int)Cg, 48)));
  VitChunk c;
  c.s0 = s0;
  c.C = live ? Cw : 0u;
  c.nroutes = c.C ? (uint32_t)__shfl(incl, (int)c.C - 1, 16) : 0u;
  c.rbase = (uint32_t)__builtin_amdgcn_mov_dpp((int)d.off, 0x150, 0xf, 0xf, false);   // row_newbcast:0
  const bool inc = (uint32_t)j < c.C;
  c.kb = inc ? d.kb : 0u;
  c.rel = inc ? incl - d.cnt : 0u;
  c.gc = d.gc;
  return c;
}

// The loads run past the chunk's last route / row without a clamp (one address per lane, the rest
// immediate offsets): a chunk starts at most one past the batch's last route or layer and reads
// <= 256 routes / 16 rows from there, inside the pools' slack (the route pools hold >= 1,024
// entries past the batch's routes, the point arrays >= 64 points past its points: ensure /
// ensure_trans_raw).  What lies past the chunk is staged but never selected.
// Round 6: the loads past the chunk's routes and rows are clamped to its last
// route / row (the same lines again) instead of reading kVitRoutes routes and 16 rows whatever the
// chunk holds -- C2 K3 moved 1.73x its algorithmic bytes.  Still one unconditional load per slot
// (a v_min, no branch, no register merge).
#ifndef RM_VIT_CLAMP
#define RM_VIT_CLAMP 0
#endif
template <bool TURN>
__device__ __forceinline__ void vit_load(const DevBatch& b, uint32_t o, const VitChunk& c, int j, VitRegs<TURN>& r) {
#if RM_VIT_CLAMP
  const uint32_t rl = c.nroutes ? c.nroutes - 1u : 0u;                  // the chunk's last route
  const uint32_t sl = c.C ? c.C * (kMaxCand / 4) - 1u : 0u;             // ... and its last row quarter
  if constexpr (TURN) {
    const double* rp = b.route_d + c.rbase;
#pragma unroll
    for (int x = 0; x < kVitRoutes / 16; ++x) r.rd[x] = rp[min((uint32_t)(16 * x + j), rl)];
  } else {
    const uint32_t* rp = b.route + c.rbase;
#pragma unroll
    for (int x = 0; x < kVitRoutes / 16; ++x) r.rv[x] = rp[min((uint32_t)(16 * x + j), rl)];
  }
  const v3_f4* src = reinterpret_cast<const v3_f4*>(b.cand_sq) + (uint64_t)(c.C ? o + c.s0 : 0u) * (kMaxCand / 4);
#pragma unroll
  for (int x = 0; x < 4; ++x) r.sv[x] = src[min((uint32_t)(16 * x + j), sl)];
#else
  if constexpr (TURN) {
    const double* rp = b.route_d + c.rbase + j;
#pragma unroll
    for (int x = 0; x < kVitRoutes / 16; ++x) r.rd[x] = rp[16 * x];
  } else {
    const uint32_t* rp = b.route + c.rbase + j;
#pragma unroll
    for (int x = 0; x < kVitRoutes / 16; ++x) r.rv[x] = rp[16 * x];
  }
  const v3_f4* src = reinterpret_cast<const v3_f4*>(b.cand_sq) + (uint64_t)(c.C ? o + c.s0 : 0u) * (kMaxCand / 4) + j;
#pragma unroll
  for (int x = 0; x < 4; ++x) r.sv[x] = src[16 * x];
#endif
}

template <bool TURN>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RM_VIT_WPE))) k_viterbi(DevBatch b) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  __shared__ VitGroup smem[4];
  const int lane = threadIdx.x;
  const int j = lane & 15, gb = lane & 48;
  VitGroup& gs = smem[lane >> 4];
  const uint32_t k = blockIdx.x * 4 + (lane >> 4);
  const bool active = k < b.T;
  const uint32_t o = active ? b.trace_off[k] : 0u, S = active ? b.n_states[k] : 0u;
  const MatchOptions op = b.opts[active ? b.trace_opt[k] : 0u];
  const double inv2s2 = 1.0 / (2.0 * (double)op.sigma_z * (double)op.sigma_z);
  const double inv_beta = 1.0 / (double)op.beta;
  const double brk = (double)op.breakage_distance;
  const double INF = __longlong_as_double(0x7ff0000000000000ll);
  // wave masks (all lanes of a group alike): the group's previous layer had candidates (pok)
  unsigned long long pok = 0ull;
  uint32_t prevK = 0;
  double cj = INF;   // cost of candidate j of the previous layer
  bool fok = false;  // the trace has ended with a chain (fK candidates, costs fcj) still to trace back
  uint32_t fK = 0;
  double fcj = INF;
  // chunk 0: describe, lay out, load; then describe chunk 1
  VitChunk cur = vit_layout(vit_cook(vit_raw_any(b, o, S, 0, j), S, 0, j), 0, S, j, gb);
  VitRegs<TURN> rg;
  vit_load<TURN>(b, o, cur, j, rg);
  VitLayerRaw dn = vit_raw_any(b, o, S, cur.C, j);
  for (;;) {
    if (__ballot(cur.s0 < S) == 0ull) break;
    const uint32_t C = cur.C, nroutes = cur.nroutes, rbase = cur.rbase;
    // ---- this chunk -> LDS (its loads were issued a chunk ago); every entry written
#pragma unroll
    for (int x = 0; x < kVitRoutes / 16; ++x) {
      if constexpr (TURN) gs.route_m[j + 16 * x] = rg.rd[x];
      else gs.route_m[j + 16 * x] = rg.rv[x] == kRouteInvalid ? INF : (double)rg.rv[x] * 0.01;
    }
#pragma unroll
    for (int x = 0; x < 4; ++x) reinterpret_cast<v3_f4*>(&gs.sq[0][0])[j + 16 * x] = rg.sv[x];
    gs.kb[j] = cur.kb;
    gs.rel[j] = cur.rel;
    gs.gc[j] = cur.gc;
    // ---- the next chunk: lay out, load (overlapping this chunk's layers); describe the one after
    {
      const uint32_t s1 = cur.s0 + C;
      cur = vit_layout(vit_cook(dn, S, s1, j), s1, S, j, gb);
      vit_load<TURN>(b, o, cur, j, rg);
      dn = vit_raw_any(b, o, S, s1 + cur.C, j);
    }
    const uint32_t s0 = cur.s0 - C;   // (cur is the next chunk from here on)
    wave_sync();
    uint32_t maxC = max(C, (uint32_t)__shfl_xor((int)C, 16));
    maxC = (uint32_t)__builtin_amdgcn_readfirstlane(max(maxC, (uint32_t)__shfl_xor((int)maxC, 32)));   // wave-uniform: a scalar loop
    // layer parameters and the first four route rows run one layer ahead of their use
    uint32_t KBn = gs.kb[0], reln = gs.rel[0];
    double gcn = gs.gc[0];
    float sqn = gs.sq[0][j];
    double rmn[8];
    {
      const double* dp = gs.route_m + reln + min((uint32_t)j, KBn ? KBn - 1u : 0u);
#pragma unroll
      for (int x = 0; x < 8; ++x) rmn[x] = dp[x * KBn];
    }
    // A live group runs every layer of the loop (maxC = C for each of them).  A finished group's
    // layers have K_B = 0: at its first chunk past the end it keeps the chain its trace ended
    // with for the final backtrace (all groups at once, after the loop) and drops prev_ok, so its
    // layers neither trigger a backtrace nor need `in` selects
    {
      const bool fin = __builtin_amdgcn_inverse_ballot_w64(__builtin_amdgcn_ballot_w64(C == 0u) & pok);
      fcj = fin ? cj : fcj;
      fK = fin ? prevK : fK;
      fok = fok | fin;
      pok &= __builtin_amdgcn_ballot_w64(C != 0u);
    }
    // chain-start flags of the chunk's layers: layer t of group g at bit 16 g + t (read back at
    // bit `lane` by the flush: lane j of group g writes layer j's flag)
    unsigned long long csm = 0ull;
    for (uint32_t t = 0; t < maxC; ++t) {
      const uint32_t KB = KBn, rel = reln;
      const double gcl = gcn;
      const float sqv = sqn;
      double rm0[8];
#pragma unroll
      for (int x = 0; x < 8; ++x) rm0[x] = rmn[x];
      {
        const uint32_t tn = min(t + 1u, (uint32_t)kVitChunk - 1u);
        KBn = gs.kb[tn]; reln = gs.rel[tn]; gcn = gs.gc[tn]; sqn = gs.sq[tn][j];
      }
      double best = INF;
      int arg = -1;
      {
        const uint32_t jj = min((uint32_t)j, KB ? KB - 1u : 0u);
        const double* dp = gs.route_m + min(rel, (uint32_t)kVitRoutes - 1u) + jj;
        vit_src<0, TURN>(best, arg, cj, rm0[0], gcl, inv_beta);
        vit_src<1, TURN>(best, arg, cj, rm0[1], gcl, inv_beta);
        vit_src<2, TURN>(best, arg, cj, rm0[2], gcl, inv_beta);
        vit_src<3, TURN>(best, arg, cj, rm0[3], gcl, inv_beta);
        if (__builtin_amdgcn_ballot_w64(prevK > 4u) != 0ull) {   // sources 4..7: read a layer ahead too
          vit_src<4, TURN>(best, arg, cj, rm0[4], gcl, inv_beta);
          vit_src<5, TURN>(best, arg, cj, rm0[5], gcl, inv_beta);
          vit_src<6, TURN>(best, arg, cj, rm0[6], gcl, inv_beta);
          vit_src<7, TURN>(best, arg, cj, rm0[7], gcl, inv_beta);
          if (__builtin_amdgcn_ballot_w64(prevK > 8u) != 0ull) {
            const uint32_t kbs = min(KB, (uint32_t)kMaxCand);
            vit_min<2, TURN>(best, arg, cj, dp, kbs, prevK, gcl, inv_beta, rm0);
          }
        }
      }
      // the next layer's first route rows, read while this layer's bookkeeping runs (read again
      // after a backtrace, which stages through route_m).  Lanes past K_B and stale parameters
      // past the chunk read other bytes of this group's VitGroup, never used: no clamps
      const double* dpn = gs.route_m + reln + j;
      const uint32_t kbn = min(KBn, (uint32_t)kMaxCand);
#pragma unroll
      for (int x = 0; x < 8; ++x) rmn[x] = dpn[x * kbn];
      // the layer's bookkeeping as wave masks on the scalar unit (each compare writes one)
      const unsigned long long vm = __builtin_amdgcn_ballot_w64(j < (int)KB);      // valid targets
      const unsigned long long hm = vm & __builtin_amdgcn_ballot_w64(arg >= 0);     // ... with a transition in
      // groups with no transition into this layer (the chain breaks there too): fold each group's
      // 16 bits onto its lowest bit, spread the groups without one back over their lanes
      unsigned long long y = hm | (hm >> 1);
      y |= y >> 2;
      y |= y >> 4;
      y |= y >> 8;
      const unsigned long long g0 = y & 0x0001000100010001ull;
      const unsigned long long stm = ~pok | __builtin_amdgcn_ballot_w64(gcl > brk) | ~((g0 << 16) - g0);   // chain starts
      const unsigned long long kbm = __builtin_amdgcn_ballot_w64(KB == 0u);
      const unsigned long long btm = pok & (kbm | stm);   // the chain that ends at s - 1 is complete
      if (btm != 0ull) {
        if (__builtin_amdgcn_inverse_ballot_w64(btm)) {
          wave_sync();
          vit_flush_m(b, gs, o + s0, t, j, csm);
          backtrace_chain(b, gs, o, s0 + t - 1, prevK, j, cj);
        }
        // the backtrace staged through route_m: bring the chunk's routes back (rare path)
        const uint32_t* rp = b.route + rbase;
        const double* rdp = b.route_d ? b.route_d + rbase : nullptr;
#pragma unroll
        for (int x = 0; x < kVitRoutes / 16; ++x) {
          const uint32_t q = (uint32_t)j + 16u * x;
          if (q < nroutes) {
            if constexpr (TURN) gs.route_m[q] = rdp[q];
            else gs.route_m[q] = rp[q] == kRouteInvalid ? INF : (double)rp[q] * 0.01;
          }
        }
        wave_sync();
#pragma unroll
        for (int x = 0; x < 8; ++x) rmn[x] = dpn[x * kbn];
      }
      const bool start = __builtin_amdgcn_inverse_ballot_w64(stm);
      const double em = __builtin_amdgcn_inverse_ballot_w64(vm) ? (double)sqv * inv2s2 : INF;
      const double nc = start ? em : best + em;
      const uint32_t bpj = __builtin_amdgcn_inverse_ballot_w64(stm | ~hm) ? 255u : (uint32_t)arg;
      reinterpret_cast<uint8_t*>(&gs.bpo[t])[j] = (uint8_t)bpj;
      csm |= (stm & 0x0001000100010001ull) << t;
      cj = nc;
      pok = ~kbm;
      prevK = KB;
    }
    wave_sync();
    vit_flush_m(b, gs, o + s0, C, j, csm);
    wave_sync();
  }
  if (fok | __builtin_amdgcn_inverse_ballot_w64(pok)) backtrace_chain(b, gs, o, S - 1, fok ? fK : prevK, j, fok ? fcj : cj);
}

// Small batches (the coalesced service: tens to hundreds of traces) take the one-wave-per-trace
// kernel: with a few waves on an empty GPU the per-layer latency is the time, and its layer
// chain is shorter (C2 traces of 600 points: 0.49 -> 0.35 ms at 38 traces, 0.38 -> 0.32 ms for
// one); large batches keep four traces per wave (fewer instructions per trace-layer, 0.75 vs
// 1.01 ms on C2's 10 k traces; at 4,096 traces 0.52 vs 0.55 ms).  RM_VIT_WAVE_MAX overrides
// the crossover.
// Round 5: one to four traces fit the batch kernel's single wave, whose layer chain is now the
// shorter one (C1's 1,000-point trace: K3 0.406 -> 0.387 ms, Match 0.72 -> 0.67 ms; a lone C2
// trace even, 0.25 ms; at 38 traces the one-wave kernel still wins, 0.27 vs 0.30 ms).
// RM_VIT_WAVE_MIN overrides that bound.
#ifndef RM_VIT_WAVE_MAX
#define RM_VIT_WAVE_MAX 4096
#endif
#ifndef RM_VIT_WAVE_MIN
#define RM_VIT_WAVE_MIN 5
#endif
void launch_viterbi(uint32_t T, hipStream_t st, const DevBatch& v) {
  static const uint32_t wave_max = [] {
    const char* e = std::getenv("RM_VIT_WAVE_MAX");
    return e && *e ? (uint32_t)std::strtoul(e, nullptr, 10) : (uint32_t)RM_VIT_WAVE_MAX;
  }();
  static const uint32_t wave_min = [] {
    const char* e = std::getenv("RM_VIT_WAVE_MIN");
    return e && *e ? (uint32_t)std::strtoul(e, nullptr, 10) : (uint32_t)RM_VIT_WAVE_MIN;
  }();
  const bool turn = v.route_d != nullptr;   // the batch has turn costs (rule 3b)
  if (T >= wave_min && T <= wave_max) {
    if (turn) hipLaunchKernelGGL(k_viterbi_w<true>, dim3(T), dim3(64), 0, st, v);
    else hipLaunchKernelGGL(k_viterbi_w<false>, dim3(T), dim3(64), 0, st, v);
    return;
  }
  if (turn) hipLaunchKernelGGL(k_viterbi<true>, dim3((T + 3) / 4), dim3(64), 0, st, v);
  else hipLaunchKernelGGL(k_viterbi<false>, dim3((T + 3) / 4), dim3(64), 0, st, v);
}

// ------------------------------------------------------------------------------------------
// k_paths wave tiers: one wave per chosen transition whose search outgrew the lane tier;
// re-run the search for (i*, j*), compute canonical predecessors and write the
// directed-edge path.  Returns false when the search outgrew the hash (next tier).
template <int H, int W = kWave>
__device__ bool paths_search_item(SearchSmem<H, true>& sm, uint4* s_src, const DevGraph& g, const DevBatch& b,
                                  uint64_t p) {
  const int lane = grp_lane<W>();
  const uint4 pi = b.pair_info[p];
  const int mode = (int)(pi.z >> 16);
  const uint32_t acc = mode_access(mode);
  const uint32_t bound = pi.x;
  const uint32_t i = (uint32_t)b.choice[p - 1], j = (uint32_t)b.choice[p];
  const uint4 b0 = b.cand_desc[(p * kMaxCand + j) * 2], b1 = b.cand_desc[(p * kMaxCand + j) * 2 + 1];
  if (lane < 2) s_src[lane] = b.cand_desc[((p - 1) * kMaxCand + i) * 2 + lane];
  grp_sync<W>();
  const uint4 a0 = s_src[0], a1 = s_src[1];
  bounded_search<H, true, W>(sm, g, mode, bound, s_src, 1, 0u,
                          SearchTargets{b.cand_desc + (p * kMaxCand + j) * 2, 1u, b.search_delta});
  if (sm.ovf) {
    grp_sync<W>();
    return false;
  }
  int combo = -1;
  const unsigned long long key = route_key(HashLabel<H, true>{sm, 0u}, a0, b0, b1, &combo);
  unsigned long long rk1, rk0;
  exit_keys(a0, bound, rk1, rk0);   // root keys of the source exits (only roots within the bound exist)
  const uint32_t n1a = a1.y, n0a = a1.x;
  if (combo >= 2) {
    // canonical predecessors: min edge id among tight in-edges of non-root nodes
    for (int h = lane; h < H; h += W) {
      const uint32_t ku = sm.key[h];
      if (ku == kEmpty) continue;
      const unsigned long long lu = sm.lab[h];
      if (lu == kKeyInf) continue;
      const uint32_t u = ku & 0x0fffffffu;
      for (uint32_t e = g.node_off[u]; e < g.node_off[u + 1]; ++e) {
        const uint4 rec = g.edges[e];
        if (!edge_ok(rec.z, acc)) continue;
        const int hv = h_find(sm, rec.x);
        if (hv < 0) continue;
        const unsigned long long lv = sm.lab[hv];
        if (lv == kKeyInf) continue;
        if ((rec.x == n1a && lv == rk1) || (rec.x == n0a && lv == rk0)) continue;
        if (lu + edge_key(rec, mode) == lv) atomicMin(&sm.pred[hv], e);
      }
    }
    grp_sync<W>();
  }
  // walk the canonical predecessors once (lane 0) into an LDS buffer that reuses the
  // frontier arrays (H u32), then copy in travel order: inline slot when short, pool else
  uint32_t* pbuf = reinterpret_cast<uint32_t*>(sm.fa);
  if (lane == 0) {
    uint32_t n = 0;
    if (combo <= 1) {
      pbuf[n++] = combo == 0 ? g.road_fwd[a0.x] : g.road_rev[a0.x];
    } else {
      pbuf[n++] = combo == 2 ? g.road_fwd[b0.x] : g.road_rev[b0.x];   // entry edge (reversed order)
      uint32_t x = combo == 2 ? b1.x : b1.y;
      for (;;) {
        const int hx = h_find(sm, x);
        if (hx < 0 || n + 2 > (uint32_t)H) { trace_fail(b, p, kErrRounds); n = 0; break; }
        const unsigned long long lx = sm.lab[hx];
        if ((x == n1a && lx == rk1) || (x == n0a && lx == rk0)) break;
        const uint32_t e = sm.pred[hx];
        if (e == kNone) { trace_fail(b, p, kErrRounds); n = 0; break; }
        pbuf[n++] = e;
        x = g.edge_src[e];
      }
      if (n) pbuf[n++] = (x == n1a) ? g.road_fwd[a0.x] : g.road_rev[a0.x];  // exit edge
    }
    uint32_t at = 0;
    if (n > (uint32_t)kInlinePath) {
      at = atomicAdd(&b.ctl[0], n);
      if ((uint64_t)at + n > b.path_cap) { atomicOr(&b.ctl[2], kErrPathOverflow); at = kNone; }
    }
    b.path_cnt[p] = n;
    b.path_off[p] = at;
    b.route_dist[p] = key_dist(key);
    b.path_sab[p] = make_uint2(a0.y, b0.y);
    sm.nf = n;
    sm.nn = at;
  }
  grp_sync<W>();
  {
    const uint32_t n = sm.nf, at = sm.nn;
    uint32_t* dst = n <= (uint32_t)kInlinePath ? b.path_inline + p * kInlinePath : (at == kNone ? nullptr : b.path_pool + at);
    if (dst)
      for (uint32_t q = lane; q < n; q += W) dst[q] = pbuf[n - 1 - q];
  }
  grp_sync<W>();
  return true;
}

// path tiers, as the route tiers: group tier <- rl_paths_b (ctl[6]) -> rl_paths_a (ctl[12]) ->
// 512 tier -> rl_routes_0 (ctl[14], free once the path lane tier has run) -> 4096 tier -> rl_paths_c
// (short_chain: the path ball tier's hand-overs, rl_routes_0 / ctl[8], as k_routes_grp's)
__global__ void __launch_bounds__(64) k_paths_grp(DevGraph g, DevBatch b, int short_chain) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  __shared__ SearchSmem<kGrpPathH, true> sm[kWave / kGrpW];
  __shared__ uint4 s_src[kWave / kGrpW][2];
  const int gi = threadIdx.x / kGrpW;
  const uint32_t n_items = short_chain ? b.ctl[8] : b.ctl[6];
  const uint32_t* list = short_chain ? b.rl_routes_0 : b.rl_paths_b;
  for (uint32_t item = blockIdx.x * (kWave / kGrpW) + gi; item < n_items; item += gridDim.x * (kWave / kGrpW)) {
    const uint32_t p = list[item];
    if (!paths_search_item<kGrpPathH, kGrpW>(sm[gi], s_src[gi], g, b, p) && grp_lane<kGrpW>() == 0)
      b.rl_paths_a[atomicAdd(&b.ctl[12], 1u)] = p;
  }
}

__global__ void __launch_bounds__(64) k_paths_wave_s(DevGraph g, DevBatch b) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  __shared__ SearchSmem<kMidH, true> sm;
  __shared__ uint4 s_src[2];
  const uint32_t n_items = b.ctl[12];
  for (uint32_t item = blockIdx.x; item < n_items; item += gridDim.x) {
    const uint32_t p = b.rl_paths_a[item];
    if (!paths_search_item<kMidH>(sm, s_src, g, b, p) && threadIdx.x == 0) b.rl_routes_0[atomicAdd(&b.ctl[14], 1u)] = p;
  }
}

__global__ void __launch_bounds__(64) k_paths_wave(DevGraph g, DevBatch b, int short_chain) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  __shared__ SearchSmem<kBigH, true> sm;
  __shared__ uint4 s_src[2];
  const uint32_t n_items = short_chain ? b.ctl[12] : b.ctl[14];
  const uint32_t* list = short_chain ? b.rl_paths_a : b.rl_routes_0;
  for (uint32_t item = blockIdx.x; item < n_items; item += gridDim.x) {
    const uint32_t p = list[item];
    if (!paths_search_item<kBigH>(sm, s_src, g, b, p) && threadIdx.x == 0) b.rl_paths_c[atomicAdd(&b.ctl[10], 1u)] = p;
  }
}

__global__ void __launch_bounds__(64) k_paths_global(DevGraph g, DevBatch b, GlobalPathSmem* scratch) {
  if (steady_abort(b)) return;   // a steady run whose pools the batch outgrew (Matcher::run_steady)
  __shared__ uint4 s_src[2];
  GlobalPathSmem& sm = scratch[blockIdx.x];
  const uint32_t n_items = b.ctl[10];
  for (uint32_t item = blockIdx.x; item < n_items; item += gridDim.x) {
    const uint32_t p = b.rl_paths_c[item];
    if (!paths_search_item<kGlobalH>(sm, s_src, g, b, p) && threadIdx.x == 0) trace_fail(b, p, kErrSearchOverflow);
  }
}

// ------------------------------------------------------------------------------------------
// K4 (segments): traversal records -> OSMLR runs -> segments (meili form_segments + the
// reporter's segment fields).  Shared pieces: the run state a segment is written from, the
// time interpolation along a transition's route, and the record-vs-previous-kept-record rule
// (merge / continue / new run); k_seg_wave below applies them to 64 records at a time.
struct RunState {
  bool open, internal;
  uint32_t sd, f_b, f_soff, l_en, l_len, l_soff, seg_len, sb, se, way_first, way_last;
  double tb, te;
  uint64_t tot, q;
};

__device__ __forceinline__ void run_close(const DevGraph& g, RunState& R, SegmentRec* out, uint32_t& n) {
  if (!R.open) return;
  const uint32_t sd = R.sd;
  const bool start_ok = R.f_b == 0 && (sd == kNone || R.f_soff == 0);
  const bool end_ok = R.l_en == R.l_len && (sd == kNone || R.l_soff + R.l_len == R.seg_len);
  SegmentRec s;
  s.segment_id = sd == kNone ? kInvalidSegmentId : g.seg_id[sd];
  s.start_time = start_ok ? R.tb : -1.0;
  s.end_time = end_ok ? R.te : -1.0;
  if (sd != kNone) s.length = (start_ok && end_ok) ? (int32_t)((R.seg_len + 50u) / 100u) : -1;
  else s.length = (int32_t)((R.tot + 50u) / 100u);
  s.queue_length = (int32_t)((R.q + 50u) / 100u);
  s.flags = (sd == kNone && R.internal ? 1u : 0u) | (sd != kNone ? 2u : 0u);
  s.begin_shape_index = R.sb;
  s.end_shape_index = R.se;
  s.seg_dense = sd;
  s.way_first = R.way_first;
  s.way_last = R.way_last;
  out[n++] = s;
  R.open = false;
}

__device__ __forceinline__ double interp_time(double ta, double tb, uint64_t x, uint64_t D) {
  if (D == 0) return ta;
  return ta + (tb - ta) * ((double)x / (double)D);
}

enum : uint8_t { kRecSkip = 0, kRecNew = 1, kRecMerged = 2 };

__device__ __forceinline__ bool same_chain(uint32_t slot_prev, uint32_t slot_next) {
  // traversal records of a chain come from consecutive transition slots; traces are
  // at least two slots apart, so this also separates traces
  return slot_next == slot_prev || slot_next == slot_prev + 1;
}

// kind / head flag of t given the previous kept record u of its chain (has_u)
__device__ __forceinline__ void flag_vs(const TravRec& t, bool has_u, const TravRec& u, uint8_t& kind, uint32_t& head) {
  if (!has_u) { kind = kRecNew; head = 1; return; }
  if (u.e == t.e && u.en == t.b) { kind = kRecMerged; head = 0; return; }
  kind = kRecNew;
  bool cont = u.sd == t.sd;
  if (cont && t.sd == kNone && ((u.slot ^ t.slot) & kTravInternal)) cont = false;
  if (cont) {
    if (u.en != u.len || t.b != 0) cont = false;
    else if (t.sd != kNone && t.soff != u.soff + u.len) cont = false;
  }
  head = cont ? 0u : 1u;
}

// ------------------------------------------------------------------------------------------
// K4, one wave per trace (k_seg_wave).  The trace's traversal records are taken 64 at a
// time, one record per lane, straight into registers: rec_slot[r] names the transition a
// record comes from (k_rec_slot), a wave scan gives its distance into the transition's route
// (the interpolated times), and the meili form_segments rules become wave-wide mask algebra
// over ballots: the previous kept record of the chain (lookback), merged / new / head flags,
// piece and run extents, and the segmented sums a run folds (total length, queue length of
// the trailing slow pieces, last differing way).  The run or piece still open at a window's
// end is carried in wave-uniform registers.  Segments of trace k land at seg_base[k] = its
// first record (a trace has no more runs than records).  No LDS, no block barrier: the
// per-trace work is independent, so the launch is as wide as the trace count.
__device__ __forceinline__ int hi_le(unsigned long long m, int i) {   // highest set bit <= i, or -1
  if (i < 0) return -1;
  const unsigned long long mm = m & ((2ull << i) - 1ull);
  return mm ? 63 - __builtin_clzll(mm) : -1;
}
__device__ __forceinline__ int lo_gt(unsigned long long m, int i) {   // lowest set bit > i, or 64
  const unsigned long long mm = m & ~((2ull << i) - 1ull);
  return mm ? __builtin_ctzll(mm) : 64;
}
__device__ __forceinline__ unsigned long long wave_incl_sum(unsigned long long v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}
// value of v in lane src (clamped to 0).  Called with every lane active: a bpermute under a
// divergent condition reads nothing from the lanes the condition switched off.
template <class T>
__device__ __forceinline__ T at_lane(T v, int src) { return __shfl(v, src < 0 ? 0 : src, 64); }

__global__ void k_rec_slot(DevBatch b, uint32_t* rec_slot) {
  if (small_abort(b)) return;   // (a steady run gated off: Matcher::run_steady)
  const uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= b.P) return;
  const uint32_t n = b.path_cnt[l], r0 = b.trav_off[l];
  for (uint32_t q = 0; q < n; ++q) rec_slot[r0 + q] = (uint32_t)l;
}

// write the segment of a run (meili form_segments' segment, run_close above)
__device__ __forceinline__ void seg_emit(const DevGraph& g, const DevBatch& b, SegmentRec* out, uint32_t f_sd, bool f_int,
                                         uint32_t f_b, uint32_t f_soff, double f_tb, uint32_t f_slot, uint32_t wf,
                                         uint32_t wl, unsigned long long tot, unsigned long long q, uint32_t l_en,
                                         uint32_t l_len, uint32_t l_soff, double l_te, uint32_t l_slot) {
  RunState R;
  R.open = true; R.sd = f_sd; R.internal = f_int;
  R.seg_len = f_sd != kNone ? g.seg_len[f_sd] : 0u;
  R.f_b = f_b; R.f_soff = f_soff; R.tb = f_tb; R.sb = b.state_orig[(f_slot & kTravSlotMask) - 1u];
  R.tot = tot; R.q = q; R.way_first = wf; R.way_last = wl;
  R.l_en = l_en; R.l_len = l_len; R.l_soff = l_soff; R.te = l_te;
  const uint32_t sl = l_slot & kTravSlotMask;
  R.se = b.state_orig[(l_slot & kTravLast) ? sl : sl - 1u];
  uint32_t n = 0;
  run_close(g, R, out, n);
}

__device__ __forceinline__ bool piece_slow(unsigned long long md, double mtb, double mte) {
  const double dt = mte - mtb;
  return dt > 0.0 && ((double)md * 0.01) / dt < kQueueSpeedMps;
}

// K4's report() epilogue (round 5: fused into k_seg_wave; report_wave below): the wave that
// formed a trace's segments reports them at once, from L2, instead of a second launch of one
// wave per trace re-reading them (k_report was 0.20 ms per 125 k C3 traces)
struct ReportArgs {
  double threshold;
  uint32_t rmask, tmask;
  uint32_t* hist;
  unsigned long long* dur;
  int on;
};
__device__ __forceinline__ ReportStats report_wave(const SegmentRec* segs, uint32_t n, bool has_pts, double end_time,
                                                   double threshold, uint32_t rmask, uint32_t tmask, ReportRec* out,
                                                   uint32_t* hist, unsigned long long* dur);

// a traversal record's transition slot and the slot's data K4 reads (k_seg_wave's prefetch)
struct K4Slot {
  uint32_t l, ns, toff, pofs, D;
  uint2 sab;
  double ta, tbs;
};
__device__ __forceinline__ K4Slot k4_slot(const DevBatch& b, uint32_t l) {
  K4Slot s;
  s.l = l;
  s.ns = b.path_cnt[l];
  s.toff = b.trav_off[l];
  s.pofs = b.path_off[l];
  s.D = b.route_dist[l];
  s.sab = b.path_sab[l];
  s.ta = b.state_time[l - 1];   // a record's slot is a transition's target: l >= 1
  s.tbs = b.state_time[l];
  return s;
}

__global__ void __launch_bounds__(64) k_seg_wave(DevGraph g, DevBatch b, const uint32_t* rec_slot, uint32_t total_arg, ReportArgs ra) {
  const uint32_t k = blockIdx.x;
  if (k >= b.T || small_abort(b)) return;
  const uint32_t total = total_arg != kNone ? total_arg : (uint32_t)b.tot[2];   // kNone: a small run's
  const int lane = threadIdx.x;
  const uint32_t o = b.trace_off[k], o1 = b.trace_off[k + 1];
  const uint32_t Rb = o < b.P ? b.trav_off[o] : total;
  const uint32_t Re = o1 < b.P ? b.trav_off[o1] : total;
  const bool bad = b.trace_err[k] != 0u;   // a failed trace forms no segments (empty pieces)
  // chain lookback carry: slot of the record before the window, and whether the last kept
  // record (lk_*) is chain-continuous up to it
  uint32_t c_slot = kNone;
  bool c_has = false;
  uint32_t lk_e = 0, lk_en = 0, lk_len = 0, lk_soff = 0, lk_sd = kNone, lk_slot = 0;
  double lk_te = 0.0;
  // the run open at the window start: head fields, folded totals, the open piece
  bool r_open = false, r_int = false;
  uint32_t r_sd = kNone, r_fb = 0, r_fsoff = 0, r_fslot = 0, r_wf = 0, r_wl = 0, r_idx = 0;
  double r_tb = 0.0, p_mtb = 0.0;
  unsigned long long r_tot = 0, r_q = 0, p_md = 0;
  unsigned long long carry_x = 0;   // route distance of the transition that straddles the window start
  uint32_t runs = 0;
  // The record build is a chain of dependent loads (record -> slot -> its transition's data ->
  // path edge -> edge record).  Its first two links run ahead: a window's slots are loaded two
  // windows early and their transition data one window early, every load unconditional at a
  // clamped record index (a clamped lane's values are never used), and the next window's data is
  // taken into registers before this window's segments are stored (loads and stores share
  // vmcnt, in issue order: a wait after the stores would wait for them too).
  const uint32_t rl = Re > 0u ? Re - 1u : 0u;
  K4Slot cur{};
  uint32_t la = 0;
  if (Rb < Re) {
    cur = k4_slot(b, rec_slot[min(Rb + (uint32_t)lane, rl)]);
    la = rec_slot[min(Rb + 64u + (uint32_t)lane, rl)];
  }
  for (uint32_t c0 = Rb; c0 < Re; c0 += 64) {
    const uint32_t n = min(64u, Re - c0);
    const bool last = c0 + n == Re;
    const bool act = (uint32_t)lane < n;
    // ---- build one traversal record per lane (seg_build_slot's arithmetic)
    const uint32_t l = cur.l;
    const uint32_t q_ld = min(c0 + (uint32_t)lane, rl) - cur.toff;
    const uint32_t q = act ? q_ld : 0u;
    const uint32_t* pe = cur.ns <= (uint32_t)kInlinePath ? b.path_inline + (uint64_t)l * kInlinePath : b.path_pool + cur.pofs;
    const uint32_t e_ld = pe[q_ld];
    const uint4 sr = g.seg_rec[e_ld];
    // the next windows' links (see above), issued behind this window's own loads
    __asm__ volatile("" : : : "memory");
    const K4Slot nxt = k4_slot(b, la);
    la = rec_slot[min(c0 + 128u + (uint32_t)lane, rl)];
    uint32_t e = 0, b0 = 0, b1 = 0, L = 0, sd = kNone, soff = 0, way = 0, slotf = 0;
    const double ta = act ? cur.ta : 0.0, tbs = act ? cur.tbs : 0.0;
    const uint32_t D = act ? cur.D : 0u;
    if (act) {
      const uint32_t ns = cur.ns;
      const uint2 sab = cur.sab;
      e = e_ld;
      L = sr.x & 0x3fffffffu;
      const bool rev = (sr.x >> 31) != 0u;
      b1 = L;
      if (q == 0) b0 = rev ? L - sab.x : sab.x;
      if (q + 1 == ns) b1 = rev ? L - sab.y : sab.y;
      if (bad) b0 = b1 = 0;
      sd = sr.y; soff = sr.z; way = sr.w;
      slotf = l | (q + 1 == ns ? kTravLast : 0u) | (((sr.x >> 30) & 1u) ? kTravInternal : 0u);
    }
    const unsigned long long w = (unsigned long long)(b1 - b0);
    const unsigned long long S = wave_incl_sum(w, lane);   // also the run / piece length prefix
    const int st = lane - (int)q;                          // lane of the transition's first record
    const unsigned long long S_st = at_lane(S, st - 1);
    unsigned long long xb = S - w - (st > 0 ? S_st : 0ull);
    if (st < 0) xb += carry_x;
    const double tbr = interp_time(ta, tbs, xb, D);
    const double ter = interp_time(ta, tbs, xb + w, D);
    // ---- flags: previous kept record of the chain, kind, run head
    const bool kept = act && b1 != b0;
    const unsigned long long K = __ballot(kept);
    const uint32_t lp = __shfl_up(l, 1, 64);
    const bool brk = act && (lane == 0 ? !(c_slot != kNone && same_chain(c_slot, l)) : !same_chain(lp, l));
    const unsigned long long BR = __ballot(brk);
    const int j = hi_le(K, lane - 1), pb = hi_le(BR, lane);
    const bool has = j >= 0 ? pb <= j : (pb < 0 && c_has);
    TravRec t, u;
    t.e = e; t.b = b0; t.en = b1; t.slot = slotf; t.sd = sd; t.soff = soff; t.len = L;
    u.e = at_lane(e, j); u.b = 0; u.en = at_lane(b1, j); u.slot = at_lane(slotf, j);
    u.sd = at_lane(sd, j); u.soff = at_lane(soff, j); u.len = at_lane(L, j);
    if (j < 0) { u.e = lk_e; u.en = lk_en; u.slot = lk_slot; u.sd = lk_sd; u.soff = lk_soff; u.len = lk_len; }
    uint8_t kind = kRecSkip;
    uint32_t head = 0;
    if (kept) flag_vs(t, has, u, kind, head);
    const unsigned long long NW = __ballot(kept && kind == kRecNew);
    const unsigned long long HD = __ballot(kept && head != 0u);
    // ---- pieces (a new record and the merged records after it) and runs (head .. next head)
    // a piece carried in closes before this window's first kept record when that starts a new
    // piece of the same run (a head closes the whole run below)
    if (r_open && K != 0ull) {
      const int fk = __builtin_ctzll(K);
      if (((NW >> fk) & 1ull) && !((HD >> fk) & 1ull)) r_q = piece_slow(p_md, p_mtb, lk_te) ? r_q + p_md : 0ull;
    }
    const int ps = hi_le(NW, lane), rs = hi_le(HD, lane);
    const unsigned long long S_ps = at_lane(S, ps - 1), S_rs = at_lane(S, rs - 1);
    const double tb_ps = at_lane(tbr, ps);
    const unsigned long long md = ps >= 0 ? S - (ps > 0 ? S_ps : 0ull) : p_md + S;
    const double mtb = ps >= 0 ? tb_ps : p_mtb;
    const int nx = lo_gt(K, lane);
    const bool next_new = nx < 64 && ((NW >> nx) & 1ull);
    const bool next_head = nx < 64 && ((HD >> nx) & 1ull);
    const bool closeP = kept && (next_new || (nx == 64 && last));
    const bool endR = kept && (next_head || (nx == 64 && last));
    const bool slow = closeP && piece_slow(md, mtb, ter);
    const unsigned long long CN = __ballot(closeP && !slow);
    const unsigned long long Qs = wave_incl_sum(closeP && slow ? md : 0ull, lane);
    // head fields of this lane's run
    const uint32_t h_way = at_lane(way, rs), h_sd = at_lane(sd, rs), h_slot = at_lane(slotf, rs);
    const uint32_t h_b = at_lane(b0, rs), h_soff = at_lane(soff, rs);
    const double h_tb = at_lane(tbr, rs);
    const uint32_t wf = rs >= 0 ? h_way : r_wf;
    const unsigned long long MW = __ballot(kept && kind == kRecNew && head == 0u && way != wf);
    // folded run state through this lane (closed pieces only for the queue length)
    const int z = hi_le(CN, lane), z2 = hi_le(MW, lane);
    const unsigned long long Q_z = at_lane(Qs, z), Q_rs = at_lane(Qs, rs - 1);
    const uint32_t way_z2 = at_lane(way, z2);
    const unsigned long long qv = (z >= 0 && z >= rs) ? Qs - Q_z : (rs >= 0 ? Qs - (rs > 0 ? Q_rs : 0ull) : r_q + Qs);
    const unsigned long long totv = rs >= 0 ? S - (rs > 0 ? S_rs : 0ull) : r_tot + S;
    const uint32_t wlv = (z2 >= 0 && z2 > rs) ? way_z2 : (rs >= 0 ? wf : r_wl);
    const uint32_t f_sd = rs >= 0 ? h_sd : r_sd;
    const uint32_t f_slot = rs >= 0 ? h_slot : r_fslot;
    const uint32_t f_b = rs >= 0 ? h_b : r_fb;
    const uint32_t f_soff = rs >= 0 ? h_soff : r_fsoff;
    const double f_tb = rs >= 0 ? h_tb : r_tb;
    const bool f_int = rs >= 0 ? (f_slot & kTravInternal) != 0u : r_int;
    // the next window's slot data into registers now, before this window's stores
    cur = nxt;
    __asm__ volatile("" : "+v"(cur.l), "+v"(cur.ns), "+v"(cur.toff), "+v"(cur.pofs), "+v"(cur.D), "+v"(cur.sab.x),
                     "+v"(cur.sab.y), "+v"(cur.ta), "+v"(cur.tbs) : : "memory");
    // the run carried in closes before this window's first kept record when that is a head
    // (or, at the trace's end, when the window keeps nothing)
    if (r_open && ((K != 0ull && ((HD >> __builtin_ctzll(K)) & 1ull)) || (K == 0ull && last))) {
      if (lane == 0) {
        const bool s0 = piece_slow(p_md, p_mtb, lk_te);
        seg_emit(g, b, b.segs + Rb + r_idx, r_sd, r_int, r_fb, r_fsoff, r_tb, r_fslot, r_wf, r_wl, r_tot,
                 s0 ? r_q + p_md : 0ull, lk_en, lk_len, lk_soff, lk_te, lk_slot);
      }
      r_open = false;
    }
    if (endR) {
      const uint32_t idx = rs >= 0 ? runs + (uint32_t)__popcll(HD & ((2ull << lane) - 1ull)) - 1u : r_idx;
      seg_emit(g, b, b.segs + Rb + idx, f_sd, f_int, f_b, f_soff, f_tb, f_slot, wf, wlv, totv, qv, b1, L, soff, ter, slotf);
    }
    runs += (uint32_t)__popcll(HD);
    if (last) break;
    // ---- carry into the next window
    if (K != 0ull) {
      const int jl = 63 - __builtin_clzll(K);
      const int rsl = __shfl(rs, jl, 64);
      if (rsl >= 0) {
        r_sd = __shfl(sd, rsl, 64); r_fslot = __shfl(slotf, rsl, 64); r_fb = __shfl(b0, rsl, 64);
        r_fsoff = __shfl(soff, rsl, 64); r_tb = __shfl(tbr, rsl, 64); r_wf = __shfl(way, rsl, 64);
        r_int = (r_fslot & kTravInternal) != 0u;
        r_idx = runs - 1u;   // the window's last head
      }
      r_open = true;
      r_tot = __shfl(totv, jl, 64);
      r_q = __shfl(qv, jl, 64);
      r_wl = __shfl(wlv, jl, 64);
      p_md = __shfl(md, jl, 64);
      p_mtb = __shfl(mtb, jl, 64);
      lk_e = __shfl(e, jl, 64); lk_en = __shfl(b1, jl, 64); lk_len = __shfl(L, jl, 64);
      lk_soff = __shfl(soff, jl, 64); lk_sd = __shfl(sd, jl, 64); lk_slot = __shfl(slotf, jl, 64);
      lk_te = __shfl(ter, jl, 64);
      c_has = jl == 63 ? true : (BR >> (jl + 1)) == 0ull;
    } else {
      c_has = c_has && BR == 0ull;
    }
    c_slot = __shfl(l, (int)n - 1, 64);
    carry_x = __shfl(xb + w, (int)n - 1, 64);
  }
  if (lane == 0) {
    b.seg_base[k] = Rb;
    b.seg_cnt[k] = runs;
  }
  if (ra.on) {
    __threadfence_block();   // this wave's segment stores are visible to its loads
    const ReportStats st = report_wave(b.segs + Rb, runs, o1 > o, o1 > o ? b.time[o1 - 1] : 0.0, ra.threshold, ra.rmask,
                                       ra.tmask, b.reps + Rb, ra.hist, ra.dur);
    if (lane == 0) {
      b.rep_cnt[k] = (uint32_t)st.n_reports;
      b.stats[k] = st;
    }
  }
}

// ------------------------------------------------------------------------------------------
// A8 k_report: reference report() per trace (py/reporter_service.py:79-179) + the batch
// filter (py/simple_reporter.py:177) + per-segment 10 km/h speed histogram.
// report() of one trace by one wave (round 4; the round-3 kernel walked a trace's segment list
// in one lane, ~0.38 ms of a 125 k-trace C3 step): 64 segments per step, one per lane.  The
// rule's sequential state becomes lane algebra: the tail trim is a ballot from the end, the
// prior of segment q is the highest segment below q that may be one (q == 0 or not internal,
// :145-147; carried across steps), each lane then decides its own report (:119-134) from the
// prior's fields, reports are compacted in segment order by a ballot prefix count, and the
// counters / "last assigned" lengths come from ballots.  The same function serves k_report and
// rm_report_segments, which the reference's own report() outputs pin (tests/golden).
__device__ __forceinline__ double shfl_d(double v, int src) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __shfl((int)(uint32_t)u, src, 64), hi = __shfl((int)(uint32_t)(u >> 32), src, 64);
  return __longlong_as_double(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ ReportStats report_wave(const SegmentRec* segs, uint32_t n, bool has_pts, double end_time,
                                                   double threshold, uint32_t rmask, uint32_t tmask, ReportRec* out,
                                                   uint32_t* hist, unsigned long long* dur) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  ReportStats st;
  st.successful_count = st.unreported_count = 0;
  st.successful_length_m = st.unreported_length_m = -1;
  st.discontinuities = st.invalid_speeds = st.invalid_times = st.unassociated = 0;
  st.shape_used = -1;
  // the tail that ends within threshold seconds of the trace's last point is not reported yet
  // (:86-92): last = the highest segment whose start is not within it
  int last = -1;
  if (has_pts) {
    for (int c0 = ((int)n - 1) & ~63; c0 >= 0; c0 -= 64) {
      const int q = c0 + lane;
      const bool keep = q < (int)n && !(end_time - segs[q].start_time < threshold);
      const uint64_t m = __ballot(keep);
      if (m) { last = c0 + 63 - __clzll(m); break; }
    }
  }
  if (last >= 0 && segs[last].begin_shape_index != 0) st.shape_used = (int32_t)segs[last].begin_shape_index;
  int carried = -1;          // the prior before this step's segments (index), -1: none yet
  double prev_end = 0.0;     // end time of the segment before this step's first
  int nrep = 0;
  for (int c0 = 0; c0 <= last; c0 += 64) {
    const int q = c0 + lane;
    const bool valid = q <= last;
    const SegmentRec& sq = segs[valid ? q : last];
    const uint32_t flags = sq.flags;
    const uint64_t sid = sq.segment_id;
    const double st0 = sq.start_time, st1 = sq.end_time;
    const bool has_id = valid && (flags & 2u) != 0u, internal = valid && (flags & 1u) != 0u;
    const double pe = shfl_d(st1, lane ? lane - 1 : 0);
    const double pend = lane ? pe : prev_end;
    const bool disc = valid && q != 0 && st0 == -1.0 && pend == -1.0;
    const bool unas = valid && !has_id && !internal;
    const uint64_t E = __ballot(valid && (!internal || q == 0));
    const uint64_t eb = E & below;
    const int pj = eb ? c0 + 63 - __clzll(eb) : carried;
    bool succ = false, unrep = false, bad_t = false, bad_v = false;
    int32_t plen = 0;
    ReportRec r;
    if (valid && pj >= 0 && !internal) {
      const SegmentRec& P = segs[pj];
      plen = P.length;
      if ((P.flags & 2u) && plen > 0) {
        const int p_lvl = (int)(P.segment_id & 7ull);
        if ((rmask >> (p_lvl + 1)) & 1u) {
          const int lvl = has_id ? (int)(sid & 7ull) : -1;
          const bool to_next = ((tmask >> (lvl + 1)) & 1u) != 0u;
          r.id = P.segment_id; r.t0 = P.start_time; r.t1 = to_next ? st0 : P.end_time;
          r.length = plen; r.queue_length = P.queue_length; r.seg_dense = P.seg_dense; r.pad = 0;
          r.next_id = (to_next && has_id) ? sid : kInvalidSegmentId;
          const double dt = r.t1 - r.t0;
          if (dt <= 0 || isinf(dt) || isnan(dt)) bad_t = true;
          else if (((double)plen / dt) * 3.6 > 160.0) bad_v = true;
          else succ = true;
        } else {
          unrep = true;
        }
      }
    }
    const uint64_t ms = __ballot(succ), mu = __ballot(unrep);
    if (succ) {
      out[nrep + __popcll(ms & below)] = r;
      const double dt = r.t1 - r.t0;
      if ((hist || dur) && r.t0 > 0 && r.t1 > 0 && dt > 0.5 && r.length > 0 && r.queue_length >= 0 &&
          r.seg_dense != kNone) {
        int bin = (int)(((double)r.length / dt) * 3.6 / 10.0);
        bin = bin > kHistBins - 1 ? kHistBins - 1 : (bin < 0 ? 0 : bin);
        if (hist) atomicAdd(&hist[(uint64_t)r.seg_dense * kHistBins + (uint32_t)bin], 1u);
        // the tile row's duration column, int(round(t1 - t0)) (py/simple_reporter.py:179;
        // Python 2 round() is half away from zero, as round()), summed per segment
        if (dur) atomicAdd(&dur[r.seg_dense], (unsigned long long)round(dt));
      }
    }
    nrep += __popcll(ms);
    st.successful_count += __popcll(ms);
    st.unreported_count += __popcll(mu);
    st.invalid_times += __popcll(__ballot(bad_t));
    st.invalid_speeds += __popcll(__ballot(bad_v));
    st.discontinuities += __popcll(__ballot(disc));
    st.unassociated += __popcll(__ballot(unas));
    const int ls = ms ? 63 - __clzll(ms) : 0, lu = mu ? 63 - __clzll(mu) : 0;
    const int32_t len_s = __shfl(plen, ls, 64), len_u = __shfl(plen, lu, 64);
    if (ms) st.successful_length_m = len_s;
    if (mu) st.unreported_length_m = len_u;
    if (E) carried = c0 + 63 - __clzll(E);
    prev_end = shfl_d(st1, 63);
  }
  st.n_reports = nrep;
  return st;
}

// report() over host-supplied segment lists (rm_report_segments): per-trace end time,
// threshold and level masks; reports of trace k start at seg_off[k]
__global__ void __launch_bounds__(64) k_report_lists(uint32_t T, const uint32_t* seg_off, const SegmentRec* segs,
                                                     const double* end_time, const double* threshold,
                                                     const uint32_t* rmask, const uint32_t* tmask, ReportRec* reps,
                                                     ReportStats* stats) {
  const uint32_t k = blockIdx.x;
  const uint32_t o = seg_off[k];
  const ReportStats st = report_wave(segs + o, seg_off[k + 1] - o, true, end_time[k], threshold[k], rmask[k], tmask[k],
                                     reps + o, nullptr, nullptr);
  if (threadIdx.x == 0) stats[k] = st;
}

// u64 totals of one or two u32 count arrays: the u32 exclusive scans that lay out routes and
// records would wrap silently past 2^32, so the host checks these totals instead of off+cnt
// u64 total of a u32 count array (four per lane, one atomic per block)
// block partials of the sum of a[0, n) (four u32 per lane), scanned by k_scan_parts
__global__ void __launch_bounds__(256) k_sum_u64(const uint32_t* a, uint64_t n, unsigned long long* part) {
  const uint64_t i = ((uint64_t)blockIdx.x * 256u + threadIdx.x) * 4u;
  unsigned long long v = 0;
  if (i + 4 <= n) {
    const uint4 q = *reinterpret_cast<const uint4*>(a + i);
    v = (unsigned long long)q.x + q.y + q.z + q.w;
  } else {
    for (uint64_t x = i; x < n; ++x) v += a[x];
  }
  block_sum2_u64(v, 0, part);
}

// ------------------------------------------------------------------------------------------
// Route-ball build on the GPU (balls.hpp; the host build is balls.cpp): one wave per node
// runs the bounded search from the node (key 0) in an LDS hash, folds the settled nodes
// into one row per incident road, and (pass 1) sizes the node's table or (pass 2) inserts
// the rows into it by linear probing.  Keys are the exact ones the host Dijkstra settles, so
// every lookup agrees with the host tables (row order inside a table may differ).  A node
// whose ball outgrows the LDS hash is reported (stats[1]) and the caller builds on the host.
constexpr int kBallSearchH = 256;
constexpr int kBallRowH = 256;
// largest table a node gets here: a power of two >= kBallSlotsPerRow x the 3/4-full row hash
constexpr uint32_t pow2_at_least(uint32_t x) { return x <= 1u ? 1u : 2u * pow2_at_least((x + 1u) / 2u); }
constexpr uint32_t kBallMaxTable = pow2_at_least(kBallSlotsPerRow * (kBallRowH * 3 / 4));
struct BallSmem {
  SearchSmem<kBallSearchH, false> s;
  uint32_t road[kBallRowH];
  unsigned long long k0[kBallRowH], k1[kBallRowH];
  uint8_t p0[kBallRowH], p1[kBallRowH];          // fill pass: the endpoints' canonical predecessor indices
  uint8_t pidx[kBallSearchH];                     // fill pass: per settled slot
  uint16_t dense[kBallRowH], order[kBallRowH];   // fill pass: occupied row slots, rows by rank
  uint16_t tslot[kBallMaxTable];                 // fill pass: the node's table (row slot per table slot)
  uint32_t used, bad;
};

__device__ __forceinline__ uint32_t table_bits_dev(uint32_t rows) {
  uint32_t bits = 1;
  while ((1ull << bits) < (unsigned long long)kBallSlotsPerRow * rows) ++bits;
  return bits;
}

// stats: [0] rows stored [1] nodes whose ball outgrew the LDS hashes [2] nodes without a table
template <bool FILL>
__global__ void __launch_bounds__(64) k_ball_build(DevGraph g, int mode, uint32_t radius, uint32_t max_keys,
                                                   const uint32_t* inc_off, const uint32_t* inc, uint32_t* bits_out,
                                                   const uint2* hdr, uint4* ent, unsigned long long* stats) {
  __shared__ BallSmem sm;
  const int lane = threadIdx.x;
  unsigned long long n_rows = 0, n_ovf = 0, n_none = 0;   // stats of this block's nodes (lane 0)
  for (uint32_t u = blockIdx.x; u < g.n_nodes; u += gridDim.x) {
    if (FILL && hdr[u].y == 0u) continue;
    bounded_search<kBallSearchH, false>(sm.s, g, mode, radius, nullptr, 0u, u);
    for (int h = lane; h < kBallRowH; h += kWave) {
      sm.road[h] = kEmpty; sm.k0[h] = kKeyInf; sm.k1[h] = kKeyInf;
      sm.p0[h] = (uint8_t)kBallPredNone; sm.p1[h] = (uint8_t)kBallPredNone;
    }
    if (lane == 0) { sm.used = 0; sm.bad = sm.s.ovf ? 2u : 0u; }
    if (FILL && g.ball_road_mask != ~0u && !sm.s.ovf) {
      // canonical predecessor of every settled node (rm_common.hpp kBallRoadBits; the host build
      // computes the same in balls.cpp pred_index): the first usable in-edge, in edge-id order,
      // from a settled node whose key plus the edge's key is the node's key
      const uint32_t acc = mode_access(mode);
      for (int h = lane; h < kBallSearchH; h += kWave) {
        const uint32_t v = sm.s.key[h];
        uint32_t pv = kBallPredNone;
        if (v != kEmpty && v != u) {
          const unsigned long long lab = sm.s.lab[h];
          const uint32_t q0 = g.in_off[v], q1 = g.in_off[v + 1];
          for (uint32_t q = q0; q < q1 && q - q0 < kBallPredNone; ++q) {
            const uint4 r = g.in_rec[q];
            const uint32_t inf = g.in_info[q];
            if (!edge_ok(inf, acc)) continue;
            const unsigned long long lu = h_label(sm.s, r.y);
            if (lu != kKeyInf && lu + make_key(r.w, time_ms_dev(r.w, mode_speed_dkph(mode, inf & 0xffffu))) == lab) {
              pv = q - q0;
              break;
            }
          }
        }
        sm.pidx[h] = (uint8_t)pv;
      }
    }
    __syncthreads();
    if (!sm.bad) {
      for (int h = lane; h < kBallSearchH; h += kWave) {
        const uint32_t v = sm.s.key[h];
        if (v == kEmpty) continue;
        const unsigned long long lab = sm.s.lab[h];
        if (!ball_key_fits(lab)) { atomicOr(&sm.bad, 1u); continue; }
        for (uint32_t q = inc_off[v]; q < inc_off[v + 1]; ++q) {
          const uint32_t r = inc[q];
          uint32_t x = (r * 2654435761u) & (kBallRowH - 1);
          int probe = 0;
          for (; probe < kBallRowH; ++probe, x = (x + 1) & (kBallRowH - 1)) {
            uint32_t cur = sm.road[x];
            if (cur == kEmpty) {
              cur = atomicCAS(&sm.road[x], kEmpty, r);
              if (cur == kEmpty && atomicAdd(&sm.used, 1u) >= (uint32_t)(kBallRowH * 3 / 4)) atomicOr(&sm.bad, 2u);
              if (cur == kEmpty) cur = r;
            }
            if (cur == r) break;
          }
          if (probe == kBallRowH) { atomicOr(&sm.bad, 2u); break; }
          if (g.road_node0[r] == v) { sm.k0[x] = lab; if (FILL) sm.p0[x] = sm.pidx[h]; }
          if (g.road_node1[r] == v) { sm.k1[x] = lab; if (FILL) sm.p1[x] = sm.pidx[h]; }
        }
      }
    }
    __syncthreads();
    const uint32_t bad = sm.bad, rows = sm.used, settled = sm.s.used;
    if (!FILL) {
      // as the host build: no table for a ball of more than max_keys nodes, rows of more than
      // 2 * max_keys roads, or a key beyond the 24-bit row fields
      uint32_t bits = 0;
      if (!bad && settled <= max_keys && rows <= 2u * max_keys) bits = table_bits_dev(rows);
      if (lane == 0) {
        bits_out[u] = bits;
        n_ovf += (bad & 2u) ? 1u : 0u;
        n_none += bits ? 0u : 1u;
        n_rows += bits ? rows : 0u;
      }
    } else {
      // Rows go in in order of their nearer endpoint's key, as the host build inserts them
      // (Dijkstra settle order): linear probing leaves the first-inserted rows at their home
      // slots, and K2 / the path walk probe near roads far more often than far ones (C4 at
      // 1000 m: K2 23.2 -> 19.8 ms against tables filled in LDS-hash order).  The table is
      // laid out in LDS by one lane, then written with coalesced stores.
      const uint2 hh = hdr[u];
      const uint32_t nslot = 1u << hh.y, mask = nslot - 1u;
      uint32_t n = 0;
      for (int h0 = 0; h0 < kBallRowH; h0 += kWave) {
        const bool has = sm.road[h0 + lane] != kEmpty;
        const unsigned long long m = __ballot(has);
        if (has) sm.dense[n + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)(h0 + lane);
        n += (uint32_t)__popcll(m);
      }
      for (uint32_t s = lane; s < nslot; s += kWave) sm.tslot[s] = 0xffffu;
      __syncthreads();
      for (uint32_t a = lane; a < n; a += kWave) {
        const uint32_t h = sm.dense[a], r = sm.road[h];
        const unsigned long long kh = min(sm.k0[h], sm.k1[h]);
        uint32_t rank = 0;
        for (uint32_t c = 0; c < n; ++c) {
          const uint32_t hq = sm.dense[c], rq = sm.road[hq];
          const unsigned long long kq = min(sm.k0[hq], sm.k1[hq]);
          rank += (kq < kh || (kq == kh && rq < r)) ? 1u : 0u;
        }
        sm.order[rank] = (uint16_t)h;
      }
      __syncthreads();
      if (lane == 0) {
        for (uint32_t q = 0; q < n; ++q) {
          const uint32_t h = sm.order[q];
          uint32_t x = ball_slot(sm.road[h], hh.y);
          while (sm.tslot[x] != 0xffffu) x = (x + 1) & mask;
          sm.tslot[x] = (uint16_t)h;
        }
      }
      __syncthreads();
      for (uint32_t s = lane; s < nslot; s += kWave) {
        const uint32_t h = sm.tslot[s];
        if (h == 0xffffu) continue;
        uint32_t y, z, w;
        ball_pack(sm.k0[h], sm.k1[h], y, z, w);
        ent[ball_row0(hh.x) + s] = make_uint4(ball_road_word(sm.road[h], sm.p0[h], sm.p1[h], g.ball_road_mask), y, z, w);
      }
    }
    __syncthreads();
  }
  // one atomic per block and counter (same-address atomics serialise across the XCDs)
  if (!FILL && lane == 0) {
    if (n_rows) atomicAdd(&stats[0], n_rows);
    if (n_ovf) atomicAdd(&stats[1], n_ovf);
    if (n_none) atomicAdd(&stats[2], n_none);
  }
}

__global__ void k_ball_entries(const uint32_t* bits, uint32_t n, unsigned long long* cnt) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u < n) cnt[u] = bits[u] ? (1ull << bits[u]) : 0ull;
}

__global__ void k_ball_hdr(const uint32_t* bits, const unsigned long long* off, uint32_t n, uint2* hdr) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u < n) hdr[u] = make_uint2((uint32_t)(off[u] >> 1), bits[u]);   // first rows are even (rm_common.hpp)
}

// keys from node `from` to both endpoints of `road` through the mode's tables, as K2 probes
// them (rm_engine_ball_lookup; all-ones when outside the ball or the node has no table)
__global__ void k_ball_lookup(DevGraph g, int mode, uint64_t n, const uint32_t* from, const uint32_t* road,
                              unsigned long long* keys, uint8_t* preds) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint2 h = g.ball_hdr[mode][from[i]];
  unsigned long long k0 = kKeyInf, k1 = kKeyInf;
  uint32_t p0 = kBallPredNone, p1 = kBallPredNone;
  if (h.y) {
    const uint4* ent = g.ball_ent[mode];
    const uint32_t rm = g.ball_road_mask;
    const uint4 e = ball_resolve(ent, h, road[i], ent[ball_row0(h.x) + ball_slot(road[i], h.y)], rm);
    if (e.x != kNone && (e.x & rm) == road[i]) {
      k0 = row_key0(e);
      k1 = row_key1(e);
      p0 = ball_pred(e.x, 0, rm);
      p1 = ball_pred(e.x, 1, rm);
    }
  }
  keys[2 * i] = k0;
  keys[2 * i + 1] = k1;
  if (preds) { preds[2 * i] = (uint8_t)p0; preds[2 * i + 1] = (uint8_t)p1; }
}

// Turn row word of endpoint `side` of row e (road r) in the table of node x (rm_common.hpp
// kTurnTMask): the canonical route x -> v walked back from v through the table's own rows -- the
// predecessor stored in the row, or when that index was not stored a scan of v's in-edges for the
// first usable tight one (as ball_pred_step) -- summing the turn at every node but x; at x the
// heading the route leaves x with.  kTurnNone when v is outside the ball or the sum does not fit.
__device__ uint32_t ball_turn_word(const DevGraph& g, int mode, uint32_t x, const uint2& h, const uint4* ent, uint32_t rm,
                                   uint4 e, uint32_t side) {
  unsigned long long kv = side ? row_key1(e) : row_key0(e);
  if (e.x == kNone || kv == kKeyInf) return kTurnNone;
  const uint32_t acc = mode_access(mode);
  const uint32_t r = e.x & rm;
  uint32_t hs = head_start(g.road_head[r], side);   // the entry edge onto r leaves v with this heading
  uint32_t v = side ? g.road_node1[r] : g.road_node0[r];
  uint32_t T = 0;
  for (uint32_t guard = 0; guard <= kBallMaxKeysHost + 1u; ++guard) {
    if (v == x) return T | hs << kTurnHeadShift;
    const uint32_t q0 = g.in_off[v];
    const uint32_t idx = ball_pred(e.x, side, rm);
    uint4 rec = make_uint4(kNone, 0u, 0u, 0u);
    if (idx < kBallPredNone) {
      rec = g.in_rec[q0 + idx];
    } else {
      for (uint32_t q = q0, q1 = g.in_off[v + 1]; q < q1; ++q) {
        const uint4 rr = g.in_rec[q];
        const uint32_t inf = g.in_info[q];
        if (!edge_ok(inf, acc)) continue;
        const uint32_t r2 = rr.z >> 1;
        const uint4 eu = ball_resolve(ent, h, r2, ent[ball_row0(h.x) + ball_slot(r2, h.y)], rm);
        const unsigned long long ku = (rr.z & 1u) ? row_key1(eu) : row_key0(eu);
        if (ku != kKeyInf && ku + make_key(rr.w, time_ms_dev(rr.w, mode_speed_dkph(mode, inf & 0xffffu))) == kv) {
          rec = rr;
          break;
        }
      }
      if (rec.x == kNone) return kTurnNone;
    }
    const uint32_t r2 = rec.z >> 1, rev = rec.z & 1u;
    const uint32_t hw = g.road_head[r2];
    T += g.turn_w[turn_degree(head_back(hw, rev), hs)];
    if (T >= kTurnNone) return kTurnNone;
    hs = head_start(hw, rev);
    v = rec.y;
    if (v == x) return T | hs << kTurnHeadShift;
    side = rev;   // the edge's source: node0 of its road when it runs forward
    e = ball_resolve(ent, h, r2, ent[ball_row0(h.x) + ball_slot(r2, h.y)], rm);
    kv = side ? row_key1(e) : row_key0(e);
    if (e.x == kNone || kv == kKeyInf) return kTurnNone;
  }
  return kTurnNone;
}

// turn rows of one mode's tables: one wave per node, lanes over its table's slots
__global__ void __launch_bounds__(64) k_ball_turns(DevGraph g, int mode, uint2* out) {
  const uint2* hp = g.ball_hdr[mode];
  const uint4* ent = g.ball_ent[mode];
  const uint32_t rm = g.ball_road_mask;
  for (uint32_t x = blockIdx.x; x < g.n_nodes; x += gridDim.x) {
    const uint2 h = hp[x];
    if (h.y == 0u) continue;
    const uint64_t r0 = ball_row0(h.x);
    for (uint32_t s = threadIdx.x; s < (1u << h.y); s += 64u) {
      const uint4 e = ent[r0 + s];
      uint2 w = make_uint2(kTurnNone, kTurnNone);
      if (e.x != kNone) {
        w.x = ball_turn_word(g, mode, x, h, ent, rm, e, 0u);
        w.y = ball_turn_word(g, mode, x, h, ent, rm, e, 1u);
      }
      out[r0 + s] = w;
    }
  }
}

__global__ void k_fill_edge_src(const uint32_t* node_off, uint32_t n_nodes, uint32_t* edge_src) {
  const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= n_nodes) return;
  for (uint32_t e = node_off[n]; e < node_off[n + 1]; ++e) edge_src[e] = n;
}

template <class T>
T* dalloc(std::vector<void*>& list, uint64_t n) {
  void* p = nullptr;
  if (n == 0) n = 1;
  const hipError_t e = hipMalloc(&p, n * sizeof(T));
  if (e == hipErrorOutOfMemory) {
    (void)hipGetLastError();   // not sticky: clear it for the caller's next call
    throw OutOfDeviceMemory("out of device memory allocating " + std::to_string(n * sizeof(T)) + " bytes");
  }
  RM_HIP(e);
  list.push_back(p);
  return (T*)p;
}

// a workspace that does not fit in HBM is a batch too large for the device (serve_policy.hpp)
template <class F>
void grow_workspace(F&& f) {
  try {
    f();
  } catch (const OutOfDeviceMemory& e) {
    throw BatchTooLarge(std::string("batch workspace does not fit in HBM: ") + e.what());
  }
}

template <class T>
T* upload(std::vector<void*>& list, const std::vector<T>& v) {
  T* p = dalloc<T>(list, v.size());
  if (!v.empty()) RM_HIP(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

}  // namespace

// ==========================================================================================
// Engine

// K1 reads every item listed in every grid cell its query box touches, so the engine may index
// the shape pieces on a finer grid than the graph file's: each cell split f x f.  Which roads
// a query finds never depends on it (a piece within the radius overlaps the box, so it is
// listed in a touched cell at any resolution); only how many items it reads does.  f in 1..4
// minimises, over 2,048 default-radius (50 m) queries centred on sampled shape pieces, the
// items read + 2 per touched cell row (a row costs two dependent offset loads).
// RM_GRID_SPLIT=f overrides.  C2/C3/C4 worlds: f = 2 (C2 19.4 -> 13.2 items per state, C4-like
// 11.9 -> 6.1; 3 and 4 list long pieces in too many cells).
uint32_t choose_grid_split(const Graph& g) {
  if (const char* e = std::getenv("RM_GRID_SPLIT")) return (uint32_t)std::min(8, std::max(1, std::atoi(e)));
  return choose_grid_split_for(g, 50.f);
}

uint32_t choose_grid_split_for(const Graph& g, float radius_m) {
  const GridIndex& gi = g.grid;
  const size_t n = gi.cell_item.size();
  if (n == 0) return 1;
  constexpr int kQ = 2048, kMaxF = 4;
  double cost[kMaxF + 1] = {};
  auto cell = [](double x, double x0, double d) { return (int64_t)std::floor((x - x0) / d); };
  std::vector<uint32_t> items;
  for (int q = 0; q < kQ; ++q) {
    const uint32_t v = gi.cell_item[(size_t)((double)q * (double)n / kQ)];
    const VertRec& A = g.verts[v];
    const VertRec& B = g.verts[v + 1];
    const float lon = 0.5f * (A.lon + B.lon), lat = 0.5f * (A.lat + B.lat);
    const float pad = radius_m * 1.01f + 0.5f;   // K1's padded box for the radius
    const float qlon = pad / meters_per_lon(lat), qlat = pad / (float)kMetersPerDegLat;
    const double b0 = (double)(lon - qlon), b1 = (double)(lon + qlon), c0 = (double)(lat - qlat), c1 = (double)(lat + qlat);
    // distinct items of the graph-grid cells the box touches: a superset of any finer grid's
    const int64_t x0 = std::max<int64_t>(0, cell(b0, gi.lon0, gi.dlon)), x1 = std::min<int64_t>(gi.ncx - 1, cell(b1, gi.lon0, gi.dlon));
    const int64_t y0 = std::max<int64_t>(0, cell(c0, gi.lat0, gi.dlat)), y1 = std::min<int64_t>(gi.ncy - 1, cell(c1, gi.lat0, gi.dlat));
    if (x0 > x1 || y0 > y1) continue;
    items.clear();
    for (int64_t y = y0; y <= y1; ++y)
      for (uint32_t it = gi.cell_off[y * gi.ncx + x0]; it < gi.cell_off[y * gi.ncx + x1 + 1]; ++it) items.push_back(gi.cell_item[it]);
    std::sort(items.begin(), items.end());
    items.erase(std::unique(items.begin(), items.end()), items.end());
    for (int f = 1; f <= kMaxF; ++f) {
      if ((uint64_t)gi.ncx * f * gi.ncy * f > 400000000ull) break;
      const double dl = gi.dlon / f, dt = gi.dlat / f;
      const int64_t X = (int64_t)gi.ncx * f, Y = (int64_t)gi.ncy * f;
      const int64_t qx0 = std::max<int64_t>(0, cell(b0, gi.lon0, dl)), qx1 = std::min<int64_t>(X - 1, cell(b1, gi.lon0, dl));
      const int64_t qy0 = std::max<int64_t>(0, cell(c0, gi.lat0, dt)), qy1 = std::min<int64_t>(Y - 1, cell(c1, gi.lat0, dt));
      double cnt = 0;
      for (uint32_t u : items) {
        const VertRec& P = g.verts[u];
        const VertRec& Q = g.verts[u + 1];
        const int64_t ix0 = cell(std::min(P.lon, Q.lon), gi.lon0, dl), ix1 = std::min(X - 1, cell(std::max(P.lon, Q.lon), gi.lon0, dl));
        const int64_t iy0 = cell(std::min(P.lat, Q.lat), gi.lat0, dt), iy1 = std::min(Y - 1, cell(std::max(P.lat, Q.lat), gi.lat0, dt));
        const int64_t ox = std::min(ix1, qx1) - std::max(ix0, qx0) + 1, oy = std::min(iy1, qy1) - std::max(iy0, qy0) + 1;
        if (ox > 0 && oy > 0) cnt += (double)(ox * oy);
      }
      cost[f] += cnt + 2.0 * (double)(qy1 - qy0 + 1);
    }
  }
  uint32_t best = 1;
  for (int f = 2; f <= kMaxF; ++f)
    if (cost[f] > 0 && cost[f] < 0.97 * cost[best]) best = (uint32_t)f;
  return best;
}

Engine::Engine(const Graph& g, int device) : device_(device), host_(g) {
  RM_HIP(hipSetDevice(device));
  ball_radius_cm_ = auto_ball_radius_cm(g);
  if (const char* r = std::getenv("RM_BALL_RADIUS_M"))
    ball_radius_cm_ = (uint32_t)std::min((double)kBallMaxRadiusCm, std::max(0.0, std::atof(r)) * 100.0);
  if (g.num_nodes() >= (1u << 28)) throw std::runtime_error("graph has too many nodes (limit 2^28)");
  dg_.node_off = upload(allocs_, g.node_off);
  dg_.edges = (const uint4*)upload(allocs_, g.edges);
  uint32_t* esrc = dalloc<uint32_t>(allocs_, g.num_edges());
  dg_.edge_src = esrc;
  {
    // in-edge CSR sorted by target, edge ids ascending within a node (canonical predecessors)
    std::vector<uint32_t> in_off(g.num_nodes() + 1, 0), in_edge(g.num_edges());
    for (uint32_t e = 0; e < g.num_edges(); ++e) in_off[g.edges[e].target + 1]++;
    for (uint32_t n = 0; n < g.num_nodes(); ++n) in_off[n + 1] += in_off[n];
    std::vector<uint32_t> fill(in_off.begin(), in_off.end() - 1);
    for (uint32_t e = 0; e < g.num_edges(); ++e) in_edge[fill[g.edges[e].target]++] = e;
    dg_.in_off = upload(allocs_, in_off);
    dg_.ball_road_mask = ball_road_mask(g.num_roads());
    dg_.in_edge = upload(allocs_, in_edge);
    // path walks read one self-contained record per in-edge: {edge, source node, road << 1 | rev,
    // length cm} + its info word (access, speed)
    std::vector<uint32_t> src(g.num_edges());
    for (uint32_t n = 0; n < g.num_nodes(); ++n)
      for (uint32_t e = g.node_off[n]; e < g.node_off[n + 1]; ++e) src[e] = n;
    std::vector<uint32_t> irec(4 * (size_t)g.num_edges()), iinf(g.num_edges());
    for (size_t q = 0; q < in_edge.size(); ++q) {
      const uint32_t e = in_edge[q];
      const EdgeRec& er = g.edges[e];
      irec[4 * q] = e; irec[4 * q + 1] = src[e]; irec[4 * q + 2] = er.road; irec[4 * q + 3] = er.len_cm;
      iinf[q] = er.info;
    }
    dg_.in_rec = (const uint4*)upload(allocs_, irec);
    dg_.in_info = upload(allocs_, iinf);
  }
  dg_.edge_seg = upload(allocs_, g.edge_seg);
  {
    // K4 reads one 16-byte record per path edge: {len_cm | reversed << 31 | internal << 30,
    // OSMLR segment, offset in segment, way id}
    std::vector<uint32_t> sr(4 * (size_t)g.num_edges());
    for (uint32_t e = 0; e < g.num_edges(); ++e) {
      const EdgeRec& r = g.edges[e];
      if (r.len_cm >= (1u << 30)) throw std::runtime_error("edge longer than 2^30 cm");
      sr[4 * (size_t)e] = r.len_cm | ((r.road & 1u) << 31) | ((r.info & kFlagInternal) ? 1u << 30 : 0u);
      sr[4 * (size_t)e + 1] = g.edge_seg[e];
      sr[4 * (size_t)e + 2] = g.edge_seg_off[e];
      sr[4 * (size_t)e + 3] = g.edge_way[e];
    }
    dg_.seg_rec = (const uint4*)upload(allocs_, sr);
  }
  dg_.edge_seg_off = upload(allocs_, g.edge_seg_off);
  dg_.edge_way = upload(allocs_, g.edge_way);
  dg_.road_node0 = upload(allocs_, g.road_node0);
  dg_.road_node1 = upload(allocs_, g.road_node1);
  dg_.road_fwd = upload(allocs_, g.road_fwd);
  dg_.road_rev = upload(allocs_, g.road_rev);
  dg_.road_len = upload(allocs_, g.road_len_cm);
  {
    // turn costs (rule 3b): each road's headings at node0 and node1 into it, as Valhalla's
    // NodeInfo holds them (heading_along: 30 m along the shape), and the turn weights
    // round(65536 exp(-d/45))
    std::vector<uint32_t> hw(g.num_roads());
    for (uint32_t r = 0; r < g.num_roads(); ++r) {
      const uint32_t a = g.road_vert_off[r], b = g.road_vert_off[r + 1] - 1, n = b - a + 1;
      const auto fwd = [&](uint32_t i, float& lon, float& lat) { lon = g.verts[a + i].lon; lat = g.verts[a + i].lat; };
      const auto rev = [&](uint32_t i, float& lon, float& lat) { lon = g.verts[b - i].lon; lat = g.verts[b - i].lat; };
      const uint32_t h0 = node_heading_deg(heading_along(fwd, n));
      const uint32_t h1 = node_heading_deg(heading_along(rev, n));
      hw[r] = h0 | h1 << 16;
    }
    dg_.road_head = upload(allocs_, hw);
    std::vector<uint32_t> tw(kTurnDegrees);
    for (int d = 0; d < kTurnDegrees; ++d) tw[d] = (uint32_t)std::lround(65536.0 * std::exp(-(double)d / 45.0));
    dg_.turn_w = upload(allocs_, tw);
  }
  dg_.verts = (const uint4*)upload(allocs_, g.verts);
  dg_.seg_id = (const unsigned long long*)upload(allocs_, g.seg_id);
  dg_.seg_len = upload(allocs_, g.seg_len_cm);
  // K1's grid: the graph's own, or each of its cells split f x f (choose_grid_split), chosen for
  // the default 50 m query; and when wider queries (a batch radius of 75 m and up) read fewer
  // items on another split, that grid too (CITY30's 100 m queries, f 1 vs 2)
  if (g.num_roads() >= (1u << 29)) throw std::runtime_error("graph has too many roads (limit 2^29)");
  grid_split_ = choose_grid_split(g);
  uint32_t alt = grid_split_;
  {
    const char* e = std::getenv("RM_GRID_ALT");   // 0: one grid (A/B)
    if (!std::getenv("RM_GRID_SPLIT") && !(e && *e == '0')) alt = choose_grid_split_for(g, 100.f);
  }
  auto build_k1_grid = [&](uint32_t f, K1Grid& out) {
    GridIndex split;
    if (f > 1) {
      split.lon0 = g.grid.lon0; split.lat0 = g.grid.lat0;
      split.dlon = g.grid.dlon / f; split.dlat = g.grid.dlat / f;
      split.ncx = g.grid.ncx * f; split.ncy = g.grid.ncy * f;
      build_grid_index(g.verts, split);
    }
    const GridIndex& gk = f > 1 ? split : g.grid;
    out.cell_off = upload(allocs_, gk.cell_off);
    // K1 reads cell items as self-contained records (no item -> vertex -> road chain)
    auto acc_of = [&](uint32_t e) { return e == kNone ? 0u : edge_access(g.edges[e].info); };
    std::vector<uint32_t> rec(8 * (size_t)gk.cell_item.size());
    for (size_t it = 0; it < gk.cell_item.size(); ++it) {
      const uint32_t v = gk.cell_item[it];
      const VertRec& A = g.verts[v];
      const VertRec& B = g.verts[v + 1];
      const uint32_t road = A.road;
      const uint32_t acc = acc_of(g.road_fwd[road]) | acc_of(g.road_rev[road]);
      uint32_t* r = rec.data() + 8 * it;
      std::memcpy(r + 0, &A.lon, 4); std::memcpy(r + 1, &A.lat, 4);
      std::memcpy(r + 2, &B.lon, 4); std::memcpy(r + 3, &B.lat, 4);
      r[4] = A.cum_cm; r[5] = B.cum_cm; r[6] = road | (acc << 29); r[7] = v;
    }
    out.cell_rec = (const uint4*)upload(allocs_, rec);
    out.lon0 = gk.lon0; out.lat0 = gk.lat0; out.dlon = gk.dlon; out.dlat = gk.dlat;
    out.ncx = gk.ncx; out.ncy = gk.ncy; out.split = f;
  };
  build_k1_grid(grid_split_, grids_[0]);
  if (alt != grid_split_) {
    build_k1_grid(alt, grids_[1]);
    n_grids_ = 2;
    grid_alt_radius_ = 75.f;
  }
  const K1Grid& gk = grids_[0];
  dg_.cell_off = gk.cell_off;
  dg_.cell_item = nullptr;   // K1 reads the self-contained records
  dg_.cell_rec = gk.cell_rec;
  {
    // per-road record: both endpoints, length and both directed edges with their info words
    std::vector<uint32_t> rr(8 * (size_t)g.num_roads());
    for (uint32_t r = 0; r < g.num_roads(); ++r) {
      const uint32_t ef = g.road_fwd[r], er = g.road_rev[r];
      uint32_t* x = rr.data() + 8 * (size_t)r;
      x[0] = g.road_node0[r]; x[1] = g.road_node1[r]; x[2] = g.road_len_cm[r]; x[3] = ef;
      x[4] = er; x[5] = ef == kNone ? 0u : g.edges[ef].info; x[6] = er == kNone ? 0u : g.edges[er].info; x[7] = 0;
    }
    dg_.road_rec = (const uint4*)upload(allocs_, rr);
    // per-node CSR ranges and per-mode relax records (K2 / path lane tiers)
    const uint32_t N = g.num_nodes(), E = g.num_edges();
    if (E >= (1u << 27)) throw std::runtime_error("graph has too many directed edges for the relax records (limit 2^27)");
    std::vector<uint32_t> nr(N);
    for (uint32_t n = 0; n < N; ++n) {
      const uint32_t deg = g.node_off[n + 1] - g.node_off[n];
      if (deg > 31) throw std::runtime_error("node out-degree above 31 is not supported by the relax records");
      nr[n] = (g.node_off[n] << 5) | deg;
    }
    dg_.node_rng = upload(allocs_, nr);
    std::vector<uint32_t> rel(4 * (size_t)E);
    for (int mode = 0; mode <= kModePedestrian; ++mode) {
      const uint32_t acc = mode_access(mode);
      for (uint32_t e = 0; e < E; ++e) {
        const EdgeRec& er = g.edges[e];
        const bool ok = (edge_access(er.info) & acc) != 0u;
        uint32_t* x = rel.data() + 4 * (size_t)e;
        x[0] = er.target;
        x[1] = ok ? er.len_cm : 0xffffffffu;
        x[2] = ok ? time_ms(er.len_cm, mode_speed_dkph(mode, edge_speed_dkph(er.info))) : 0u;
        x[3] = nr[er.target];
      }
      dg_.relax[mode] = (const uint4*)upload(allocs_, rel);
    }
  }
  dg_.lon0 = gk.lon0; dg_.lat0 = gk.lat0; dg_.dlon = gk.dlon; dg_.dlat = gk.dlat;
  dg_.ncx = gk.ncx; dg_.ncy = gk.ncy;
  {
    // locality order (k_loc_count): the K1 grid coarsened 2^shift x 2^shift into at most 64 x 64
    // region buckets (kLocBuckets), on by default on graphs of >= kLocalityNodes nodes
    // (RM_LOCALITY_NODES overrides), where the route tables and cell records outgrow the L2s
    uint32_t sh = 0;
    while (((gk.ncx - 1) >> sh) >= 64u || ((gk.ncy - 1) >> sh) >= 64u) ++sh;
    locality_shift_ = sh;
    locality_bits_ = (gk.ncx > 1 || gk.ncy > 1) ? kLocBucketBits : 0u;
    const char* ln = std::getenv("RM_LOCALITY_NODES");
    const uint64_t min_nodes = ln && *ln ? std::strtoull(ln, nullptr, 10) : kLocalityNodes;
    locality_default_ = locality_bits_ > 0 && (uint64_t)g.num_nodes() >= min_nodes;
  }
  dg_.n_nodes = g.num_nodes(); dg_.n_edges = g.num_edges(); dg_.n_segments = g.num_segments();
  if (g.num_nodes()) {
    hipLaunchKernelGGL(k_fill_edge_src, dim3((g.num_nodes() + 255) / 256), dim3(256), 0, 0, dg_.node_off,
                       g.num_nodes(), esrc);
    RM_HIP(hipGetLastError());
  }
  RM_HIP(hipDeviceSynchronize());
}

void Engine::k1_grid(float radius_m, DevGraph& g) const {
  const K1Grid& k = (n_grids_ > 1 && radius_m >= grid_alt_radius_) ? grids_[1] : grids_[0];
  g.cell_off = k.cell_off; g.cell_rec = k.cell_rec;
  g.lon0 = k.lon0; g.lat0 = k.lat0; g.dlon = k.dlon; g.dlat = k.dlat;
  g.ncx = k.ncx; g.ncy = k.ncy;
}

Engine::~Engine() {
  (void)hipSetDevice(device_);
  for (void* p : allocs_) (void)hipFree(p);
}

DevGraph Engine::dev_snapshot() const {
  std::lock_guard<std::mutex> lk(ball_mu_);
  return dg_;
}

void Engine::set_ball_radius(uint32_t radius_cm) {
  std::lock_guard<std::mutex> lk(ball_mu_);
  ball_radius_cm_ = radius_cm;
}

uint32_t Engine::mode_ball_radius(int mode) const {
  std::lock_guard<std::mutex> lk(ball_mu_);
  return (mode >= 0 && mode <= kModePedestrian && ((dg_.ball_mask >> mode) & 1u)) ? dg_.ball_radius[mode] : 0u;
}

void Engine::ball_stats(int mode, double* out4) const {
  std::lock_guard<std::mutex> lk(ball_mu_);
  for (int i = 0; i < 4; ++i) out4[i] = (mode >= 0 && mode <= kModePedestrian) ? ball_info_[mode][i] : 0.0;
}

// Route balls of every mode in mode_mask that has none yet.  Each mode gets the largest radius
// at or below the engine's (ladder: balls.hpp kBallRadii) whose sampled tables fit what is left
// of the memory granted to tables (ball_total_budget of the device's HBM, less what earlier modes
// took, and the free HBM less a reserve) and the per-mode budget; a build that still comes out
// too large steps down again; a mode nothing fits runs its transitions in the search tiers.
// auto and bus route identically and share one build (ball_twin_mode).
void Engine::ensure_balls(uint32_t mode_mask) {
  std::lock_guard<std::mutex> lk(ball_mu_);
  if (ball_radius_cm_ == 0 || host_.num_nodes() == 0) return;
  const uint32_t todo = mode_mask & ~ball_built_ & 0x1fu;
  if (!todo) return;
  RM_HIP(hipSetDevice(device_));
  const int threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  // small balls (country graphs at moderate radii: millions of nodes, tens of nodes per ball)
  // are built on the GPU; env RM_BALL_BUILD=host|gpu forces one
  const char* how = std::getenv("RM_BALL_BUILD");
  uint32_t max_keys = kBallMaxKeys;   // env RM_BALL_MAX_KEYS: tuning / tests of the no-table path
  if (const char* e = std::getenv("RM_BALL_MAX_KEYS")) max_keys = (uint32_t)std::max(1, std::atoi(e));
  constexpr uint64_t kReserve = 4ull << 30;   // HBM kept free for the first workspaces
  for (int mode = 0; mode <= kModePedestrian; ++mode) {
    if (!((todo >> mode) & 1u)) continue;
    const uint32_t bit = 1u << mode;
    const int tw = ball_twin_mode(mode);
    if (tw >= 0 && ((ball_built_ >> tw) & 1u)) {   // identical tables: share them
      dg_.ball_hdr[mode] = dg_.ball_hdr[tw];
      dg_.ball_ent[mode] = dg_.ball_ent[tw];
      dg_.ball_radius[mode] = dg_.ball_radius[tw];
      if ((dg_.ball_mask >> tw) & 1u) dg_.ball_mask |= bit;
      for (int i = 0; i < 4; ++i) ball_info_[mode][i] = ball_info_[tw][i];
      ball_gpu_ |= ((ball_gpu_ >> tw) & 1u) << mode;
      ball_built_ |= bit;
      continue;
    }
    size_t hbm_free = 0, hbm_total = 0;
    RM_HIP(hipMemGetInfo(&hbm_free, &hbm_total));
    const uint64_t total_cap = ball_total_budget(hbm_total);
    uint64_t avail = std::min<uint64_t>(ball_mode_budget(), total_cap > ball_bytes_ ? total_cap - ball_bytes_ : 0);
    avail = std::min<uint64_t>(avail, hbm_free > kReserve ? hbm_free - kReserve : 0);
    BallSample bs;
    uint32_t r = fit_ball_radius_cm(host_, mode, ball_radius_cm_, avail, &bs);
    bool built = false;
    for (; r && !built; r = next_ball_radius_cm(r)) {
      const double nodes = sample_balls(host_, r, kBallMaxKeysHost, mode).nodes;
      const bool try_gpu = how ? std::strcmp(how, "gpu") == 0 : nodes <= 48.0 && host_.num_nodes() >= 100000;
      try {
        if (try_gpu && build_balls_gpu(mode, r, max_keys, avail)) { built = true; break; }
        BallTables bt;
        build_balls(host_, mode, r, max_keys, threads, bt, avail / 16);
        std::vector<void*> tmp;   // both arrays or neither
        struct Free { std::vector<void*>& l; ~Free() { for (void* p : l) (void)hipFree(p); } } fr{tmp};
        const uint2* hdr = (const uint2*)upload(tmp, bt.hdr);
        const uint4* ent = (const uint4*)upload(tmp, bt.ent);
        allocs_.insert(allocs_.end(), tmp.begin(), tmp.end());
        tmp.clear();
        dg_.ball_hdr[mode] = hdr;
        dg_.ball_ent[mode] = ent;
        dg_.ball_radius[mode] = bt.radius_cm;
        dg_.ball_mask |= bit;
        ball_bytes_ += (uint64_t)bt.ent.size() * 4;
        ball_info_[mode][0] = (double)bt.n_keys;
        ball_info_[mode][1] = (double)(bt.ent.size() / 4);
        ball_info_[mode][2] = (double)bt.n_skipped;
        ball_info_[mode][3] = bt.build_ms;
        built = true;
      } catch (const BallsTooLarge&) {
        // the tables came out larger than sampled: the next radius down
      } catch (const OutOfDeviceMemory&) {
        // the free HBM moved under us (another matcher's workspace): the next radius down
      }
    }
    if (!built) {   // no tables for this mode: every transition of it runs in the search tiers
      dg_.ball_radius[mode] = 0;
      for (int i = 0; i < 4; ++i) ball_info_[mode][i] = 0.0;
    }
    ball_built_ |= bit;
  }
  RM_HIP(hipDeviceSynchronize());
}

// Turn rows (rule 3b, k_ball_turns) of every mode in mode_mask whose tables are built: 8 bytes per
// table slot, parallel to ball_ent, built on the GPU the first time a batch with turn costs needs
// them.  A mode they do not fit (free HBM less a reserve) keeps none: its transitions with turn
// costs run in the search tiers.  auto and bus share them as they share the tables.
void Engine::ensure_turn_rows(uint32_t mode_mask) {
  std::lock_guard<std::mutex> lk(ball_mu_);
  const uint32_t todo = mode_mask & dg_.ball_mask & ~turn_tried_ & 0x1fu;
  if (!todo) return;
  RM_HIP(hipSetDevice(device_));
  constexpr uint64_t kReserve = 4ull << 30;
  for (int mode = 0; mode <= kModePedestrian; ++mode) {
    if (!((todo >> mode) & 1u)) continue;
    const uint32_t bit = 1u << mode;
    turn_tried_ |= bit;
    const int tw = ball_twin_mode(mode);
    if (tw >= 0 && ((dg_.ball_turn_mask >> tw) & 1u) && dg_.ball_ent[tw] == dg_.ball_ent[mode]) {
      dg_.ball_turn[mode] = dg_.ball_turn[tw];
      dg_.ball_turn_mask |= bit;
      continue;
    }
    const uint64_t slots = (uint64_t)ball_info_[mode][1];
    size_t hbm_free = 0, hbm_total = 0;
    RM_HIP(hipMemGetInfo(&hbm_free, &hbm_total));
    if (slots == 0 || slots * sizeof(uint2) + kReserve > hbm_free) continue;
    uint2* rows = nullptr;
    try {
      std::vector<void*> tmp;
      rows = dalloc<uint2>(tmp, slots);
    } catch (const OutOfDeviceMemory&) {
      continue;
    }
    const auto t0 = std::chrono::steady_clock::now();
    DevGraph g = dg_;
    hipLaunchKernelGGL(k_ball_turns, dim3(std::min<uint32_t>(std::max(1u, host_.num_nodes()), 65536u)), dim3(64), 0, 0, g,
                       mode, rows);
    RM_HIP(hipGetLastError());
    RM_HIP(hipDeviceSynchronize());
    allocs_.push_back(rows);
    dg_.ball_turn[mode] = rows;
    dg_.ball_turn_mask |= bit;
    ball_bytes_ += slots * sizeof(uint2);
    turn_ms_[mode] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
}

// GPU route-ball build of one mode at radius_cm (k_ball_build); false (nothing changed) when
// some ball outgrew the kernel's LDS hashes, and the caller builds on the host.  Throws
// BallsTooLarge, allocating nothing, when the tables need more than avail_bytes (or rows
// beyond kBallMaxRows).  Called under ball_mu_.
bool Engine::build_balls_gpu(int mode, uint32_t radius_cm, uint32_t max_keys, uint64_t avail_bytes) {
  const auto t0 = std::chrono::steady_clock::now();
  const uint32_t N = host_.num_nodes();
  std::vector<uint32_t> inc_off, inc;
  road_incidence(host_, inc_off, inc);
  std::vector<void*> tmp;
  struct Free { std::vector<void*>& l; ~Free() { for (void* p : l) (void)hipFree(p); } } fr{tmp};
  const uint32_t* d_inc_off = upload(tmp, inc_off);
  const uint32_t* d_inc = upload(tmp, inc);
  uint32_t* d_bits = dalloc<uint32_t>(tmp, N);
  unsigned long long* d_cnt = dalloc<unsigned long long>(tmp, N);
  unsigned long long* d_off = dalloc<unsigned long long>(tmp, N);
  unsigned long long* d_stats = dalloc<unsigned long long>(tmp, 4);
  RM_HIP(hipMemset(d_stats, 0, 4 * sizeof(unsigned long long)));
  DevGraph g = dg_;
  const uint32_t grid = std::min<uint32_t>(N, 16384);
  hipLaunchKernelGGL(k_ball_build<false>, dim3(grid), dim3(64), 0, 0, g, mode, radius_cm, max_keys, d_inc_off,
                     d_inc, d_bits, (const uint2*)nullptr, (uint4*)nullptr, d_stats);
  hipLaunchKernelGGL(k_ball_entries, dim3((N + 255) / 256), dim3(256), 0, 0, d_bits, N, d_cnt);
  size_t tb = 0;
  RM_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, d_cnt, d_off, (int)N, (hipStream_t)0));
  void* d_tmp = dalloc<char>(tmp, tb);
  RM_HIP(hipcub::DeviceScan::ExclusiveSum(d_tmp, tb, d_cnt, d_off, (int)N, (hipStream_t)0));
  unsigned long long st[4], last[2];
  RM_HIP(hipMemcpy(st, d_stats, sizeof st, hipMemcpyDeviceToHost));
  RM_HIP(hipMemcpy(&last[0], d_off + (N - 1), 8, hipMemcpyDeviceToHost));
  RM_HIP(hipMemcpy(&last[1], d_cnt + (N - 1), 8, hipMemcpyDeviceToHost));
  if (st[1]) return false;   // a ball outgrew the LDS hashes: the host build takes the mode
  const uint64_t total = last[0] + last[1];
  if (total > kBallMaxRows || total * 16 > avail_bytes)
    throw BallsTooLarge("route balls too large for their budget; lower the radius");
  // header and rows join the engine's allocations only once both are filled
  uint2* d_hdr = dalloc<uint2>(tmp, N);
  uint4* d_ent = dalloc<uint4>(tmp, total);
  hipLaunchKernelGGL(k_ball_hdr, dim3((N + 255) / 256), dim3(256), 0, 0, d_bits, d_off, N, d_hdr);
  RM_HIP(hipMemset(d_ent, 0xff, total * sizeof(uint4)));
  hipLaunchKernelGGL(k_ball_build<true>, dim3(grid), dim3(64), 0, 0, g, mode, radius_cm, max_keys, d_inc_off,
                     d_inc, d_bits, (const uint2*)d_hdr, d_ent, d_stats);
  RM_HIP(hipGetLastError());
  RM_HIP(hipDeviceSynchronize());
  tmp.erase(std::remove(tmp.begin(), tmp.end(), (void*)d_hdr), tmp.end());
  tmp.erase(std::remove(tmp.begin(), tmp.end(), (void*)d_ent), tmp.end());
  allocs_.push_back(d_hdr);
  allocs_.push_back(d_ent);
  dg_.ball_hdr[mode] = d_hdr;
  dg_.ball_ent[mode] = d_ent;
  dg_.ball_radius[mode] = radius_cm;
  dg_.ball_mask |= 1u << mode;
  ball_bytes_ += total * 16;
  ball_info_[mode][0] = (double)st[0];
  ball_info_[mode][1] = (double)total;
  ball_info_[mode][2] = (double)st[2];
  ball_info_[mode][3] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  ball_gpu_ |= 1u << mode;
  return true;
}

void Engine::ball_lookup(int mode, uint64_t n, const uint32_t* from, const uint32_t* road, uint64_t* keys,
                         uint8_t* preds) {
  std::lock_guard<std::mutex> lk(ball_mu_);
  RM_HIP(hipSetDevice(device_));
  for (uint64_t i = 0; i < n; ++i) {
    keys[2 * i] = keys[2 * i + 1] = kKeyInf;
    if (preds) preds[2 * i] = preds[2 * i + 1] = (uint8_t)kBallPredNone;
    if (from[i] >= host_.num_nodes() || road[i] >= host_.num_roads()) throw std::runtime_error("node or road out of range");
  }
  if (!((ball_built_ >> mode) & 1u) || n == 0) return;
  std::vector<void*> tmp;
  struct Free { std::vector<void*>& l; ~Free() { for (void* p : l) (void)hipFree(p); } } fr{tmp};
  uint32_t* d_from = dalloc<uint32_t>(tmp, n);
  uint32_t* d_road = dalloc<uint32_t>(tmp, n);
  unsigned long long* d_keys = dalloc<unsigned long long>(tmp, 2 * n);
  uint8_t* d_pred = preds ? dalloc<uint8_t>(tmp, 2 * n) : nullptr;
  RM_HIP(hipMemcpy(d_from, from, n * 4, hipMemcpyHostToDevice));
  RM_HIP(hipMemcpy(d_road, road, n * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_ball_lookup, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, dg_, mode, n, d_from, d_road,
                     d_keys, d_pred);
  RM_HIP(hipGetLastError());
  RM_HIP(hipMemcpy(keys, d_keys, 2 * n * 8, hipMemcpyDeviceToHost));
  if (preds) RM_HIP(hipMemcpy(preds, d_pred, 2 * n, hipMemcpyDeviceToHost));
}

// ==========================================================================================
// Workspace / Matcher

Workspace::~Workspace() { release(); }
void Workspace::release() {
  for (void* p : allocs) (void)hipFree(p);
  allocs.clear();
  cap_points = cap_traces = cap_trans = cap_path = cap_opts = cap_segs = cap_src = cap_sort = cap_turn = 0;
  perm = loc_cursor = pcnt = nullptr;
  route_d = nullptr;
  walk = nullptr;
  cap_walk = 0;
  loc_key = nullptr;
}

Matcher::Matcher(Engine* e) : eng_(e) {
  RM_HIP(hipSetDevice(e->device()));
  RM_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  if (const char* lv = std::getenv("RM_LOCALITY"); lv && *lv) locality_ = std::max(-1, std::min(2, std::atoi(lv)));
}

void Matcher::ensure_sort(uint64_t n) {
  grow_workspace([&] {
    Workspace& w = ws_;
    if (n <= w.cap_sort && w.perm) return;
    for (void** q : {(void**)&w.perm, (void**)&w.loc_key, (void**)&w.loc_cursor, (void**)&w.pcnt}) {
      if (*q) {
        (void)hipFree(*q);
        w.allocs.erase(std::find(w.allocs.begin(), w.allocs.end(), *q));
      }
      *q = nullptr;
    }
    w.cap_sort = 0;
    const uint64_t c = std::max<uint64_t>(n, w.cap_points);
    if (c >= (uint64_t)INT32_MAX) throw BatchTooLarge("batch too large for the locality sort");
    std::vector<void*>& L = w.allocs;
    w.perm = dalloc<uint32_t>(L, c);
    w.loc_key = dalloc<uint16_t>(L, c);                 // region bucket per slot
    w.loc_cursor = dalloc<uint32_t>(L, kLocBuckets + 1);  // bucket counts -> cursors
    w.pcnt = dalloc<uint32_t>(L, c);
    w.cap_sort = c;
  });
}

Matcher::~Matcher() {
  (void)hipSetDevice(eng_->device());
  if (stream_) (void)hipStreamSynchronize(stream_);
  for (auto& ev : pending_) { (void)hipEventDestroy(ev.a); (void)hipEventDestroy(ev.b); }
  for (auto& ev : free_ev_) { (void)hipEventDestroy(ev.a); (void)hipEventDestroy(ev.b); }
  ws_.release();
  if (dl_dev_) (void)hipFree(dl_dev_);
  if (dl_host_) (void)hipHostFree(dl_host_);
  for (void* q : {(void*)jdev_, jspan_, (void*)jflag_, jtsp_})
    if (q) (void)hipFree(q);
  if (stream_) (void)hipStreamDestroy(stream_);
  if (hctl_) (void)hipHostFree(hctl_);
  if (hpack_) (void)hipHostFree(hpack_);
  if (dpack_) (void)hipFree(dpack_);
  if (hoff_) (void)hipHostFree(hoff_);
}

void Matcher::ensure(uint64_t points, uint32_t traces, uint32_t nopts) {
  grow_workspace([&] {
    Workspace& w = ws_;
    if (points <= w.cap_points && traces <= w.cap_traces && nopts <= w.cap_opts && w.ctl) return;
    // grow everything sized by points/traces (trans/path pools are grown separately)
    // grow by half again at least: a coalescing service sees batch sizes creep upwards, and each
    // regrowth frees and reallocates the whole workspace (hipFree synchronises the device) --
    // growing to each new maximum exactly cost a ~70 ms stall per new maximum (svc_client_probe)
    const uint64_t keep_trans = w.cap_trans, keep_path = w.cap_path, keep_segs = w.cap_segs, keep_src = w.cap_src;
    // the grown capacities first; when they do not fit in HBM but the batch's own sizes might, the
    // exact sizes (a batch that fits must not fail because the previous one was large)
    const uint64_t gp = std::max<uint64_t>(points, w.cap_points + w.cap_points / 2) + 64;
    const uint64_t gt = std::max<uint64_t>(traces, w.cap_traces + w.cap_traces / 2) + 16;
    const uint64_t go = std::max<uint64_t>(nopts, w.cap_opts + w.cap_opts / 2) + 4;
    try {
      alloc_points(gp, gt, go, keep_trans, keep_path, keep_segs, keep_src);
    } catch (const OutOfDeviceMemory&) {
      if (gp == points + 64 && gt == traces + 16 && go == nopts + 4) throw;
      alloc_points(points + 64, traces + 16, nopts + 4, 1, 1, 1, 1);
    }
  });
}

void Matcher::alloc_points(uint64_t cp, uint64_t ct, uint64_t co, uint64_t keep_trans, uint64_t keep_path,
                           uint64_t keep_segs, uint64_t keep_src) {
  {
    Workspace& w = ws_;
    w.release();
    // test hook: a workspace of more than RM_TEST_WS_POINTS_LIMIT points fails as out of memory
    // (tests/test_gpu_isolation.py: the grown size fails, the batch's own size must not)
    if (const char* lim = std::getenv("RM_TEST_WS_POINTS_LIMIT"); lim && *lim && cp > std::strtoull(lim, nullptr, 10))
      throw OutOfDeviceMemory("workspace above RM_TEST_WS_POINTS_LIMIT");
    std::vector<void*>& L = w.allocs;
    w.trace_off = dalloc<uint32_t>(L, ct + 1);
    w.lon = dalloc<float>(L, cp); w.lat = dalloc<float>(L, cp); w.time = dalloc<double>(L, cp);
    w.acc = dalloc<float>(L, cp); w.opts = dalloc<MatchOptions>(L, co); w.trace_opt = dalloc<uint32_t>(L, ct);
    w.slot_trace = dalloc<uint32_t>(L, cp); w.n_states = dalloc<uint32_t>(L, ct); w.state_orig = dalloc<uint32_t>(L, cp);
    w.state_time = dalloc<double>(L, cp);
    w.cand_n = dalloc<uint8_t>(L, cp); w.cand_desc = dalloc<uint4>(L, cp * kMaxCand * 2);
    w.cand_sq = dalloc<float>(L, cp * kMaxCand); w.pair_info = dalloc<uint4>(L, cp);
    w.trans_cnt = dalloc<uint32_t>(L, cp); w.trans_off = dalloc<uint32_t>(L, cp); w.gc = dalloc<double>(L, cp);
    w.src_cnt = dalloc<uint32_t>(L, cp); w.src_off = dalloc<uint32_t>(L, cp);
    w.choice = dalloc<int8_t>(L, cp); w.chain_start = dalloc<uint8_t>(L, cp); w.bp = dalloc<uint8_t>(L, cp * kMaxCand);
    w.path_off = dalloc<uint32_t>(L, cp); w.path_cnt = dalloc<uint32_t>(L, cp); w.route_dist = dalloc<uint32_t>(L, cp);
    w.path_sab = dalloc<uint2>(L, cp);
    w.path_inline = dalloc<uint32_t>(L, cp * kInlinePath);
    w.trav_off = dalloc<uint32_t>(L, cp);
    w.seg_base = dalloc<uint32_t>(L, ct); w.seg_cnt = dalloc<uint32_t>(L, ct);
    w.rep_cnt = dalloc<uint32_t>(L, ct); w.stats = dalloc<ReportStats>(L, ct);
    w.ctl = dalloc<uint32_t>(L, kCtlWords);
    w.rl_paths_a = dalloc<uint32_t>(L, cp); w.rl_paths_b = dalloc<uint32_t>(L, cp);
    w.rl_cand = dalloc<uint32_t>(L, cp);
    w.rl_paths_c = dalloc<uint32_t>(L, cp);
    w.trace_err = dalloc<uint32_t>(L, ct);
    w.tot64 = dalloc<unsigned long long>(L, 4);
    w.tot_part = dalloc<unsigned long long>(L, 2 * ((cp + 255) / 256) + 2);
    w.cap_points = cp; w.cap_traces = ct; w.cap_opts = co;
    w.gsearch = nullptr;
    w.route = nullptr; w.route_d = nullptr; w.cap_turn = 0; w.walk = nullptr; w.cap_walk = 0; w.rl_routes_a = nullptr; w.rl_routes_b = nullptr; w.rl_routes_0 = nullptr; w.rl_routes_c = nullptr; w.path_pool = nullptr; w.segs = nullptr; w.reps = nullptr; w.src_item = nullptr; w.rec_slot = nullptr;
    w.cap_trans = 0; w.cap_path = 0; w.cap_segs = 0; w.cap_src = 0;
    ensure_trans_raw(std::max<uint64_t>(keep_trans, 1), std::max<uint64_t>(keep_src, 1));
    ensure_path_raw(std::max<uint64_t>(keep_path, cp / 8 + 1024));
    ensure_segs_raw(std::max<uint64_t>(keep_segs, cp / 2 + 1024));
  }
}

static void free_one(Workspace& w, void* q) {
  if (!q) return;
  (void)hipFree(q);
  w.allocs.erase(std::find(w.allocs.begin(), w.allocs.end(), q));
}

void Matcher::ensure_trans(uint64_t n, uint64_t n_src) { grow_workspace([&] { ensure_trans_raw(n, n_src); }); }
void Matcher::ensure_path(uint64_t n) { grow_workspace([&] { ensure_path_raw(n); }); }
void Matcher::ensure_segs(uint64_t n) { grow_workspace([&] { ensure_segs_raw(n); }); }

// route_d (the transitions' distance terms with turn costs, K2 -> K3) for batches with turn costs:
// sized with route, allocated the first time a batch needs it
void Matcher::ensure_turns() {
  grow_workspace([&] {
    Workspace& w = ws_;
    const uint64_t want_walk = (w.cap_src / kK2Items + 2) * (kWalkPerBlock + 1);
    if (w.route_d && w.cap_turn >= w.cap_trans && w.cap_walk >= want_walk) return;
    free_one(w, w.route_d);
    free_one(w, w.walk);
    w.route_d = nullptr;
    w.walk = nullptr;
    w.cap_turn = 0;
    w.cap_walk = 0;
    w.route_d = dalloc<double>(w.allocs, w.cap_trans);
    w.cap_turn = w.cap_trans;
    // one region per K2 block of the item pool: a count and kWalkPerBlock entries
    w.cap_walk = want_walk;
    w.walk = dalloc<uint32_t>(w.allocs, w.cap_walk);
  });
}

void Matcher::ensure_trans_raw(uint64_t n, uint64_t n_src) {
  {
    Workspace& w = ws_;
    if (!(n <= w.cap_trans && w.route)) {
      free_one(w, w.route);
      free_one(w, w.route_d);
      free_one(w, w.walk);
      w.route = nullptr;
      w.route_d = nullptr;
      w.walk = nullptr;
      w.cap_trans = 0;
      w.cap_turn = 0;
      w.cap_walk = 0;
      const uint64_t c = n + n / 4 + 1024;
      w.route = dalloc<uint32_t>(w.allocs, c);
      w.cap_trans = c;
    }
    if (!(n_src <= w.cap_src && w.src_item)) {
      for (uint32_t** q : {&w.src_item, &w.rl_routes_a, &w.rl_routes_b, &w.rl_routes_0, &w.rl_routes_c}) {
        free_one(w, *q);
        *q = nullptr;
      }
      w.cap_src = 0;
      const uint64_t c = n_src + n_src / 4 + 1024;
      w.src_item = dalloc<uint32_t>(w.allocs, c);
      w.rl_routes_a = dalloc<uint32_t>(w.allocs, c);   // overflow lists hold (pair, source) items
      w.rl_routes_b = dalloc<uint32_t>(w.allocs, c);
      w.rl_routes_0 = dalloc<uint32_t>(w.allocs, c);
      w.rl_routes_c = dalloc<uint32_t>(w.allocs, c);
      w.cap_src = c;
    }
  }
}

void Matcher::ensure_path_raw(uint64_t n) {
  {
    Workspace& w = ws_;
    if (n <= w.cap_path && w.path_pool) return;
    free_one(w, w.path_pool);
    w.path_pool = nullptr;
    w.cap_path = 0;
    const uint64_t c = n + n / 4 + 1024;
    w.path_pool = dalloc<uint32_t>(w.allocs, c);
    w.cap_path = c;
  }
}

void Matcher::ensure_segs_raw(uint64_t n) {
  {
    Workspace& w = ws_;
    if (n <= w.cap_segs && w.segs) return;
    for (void** q : {(void**)&w.segs, (void**)&w.reps, (void**)&w.rec_slot}) {
      free_one(w, *q);
      *q = nullptr;
    }
    w.cap_segs = 0;
    const uint64_t c = n + n / 4 + 1024;
    w.segs = dalloc<SegmentRec>(w.allocs, c);
    w.reps = dalloc<ReportRec>(w.allocs, c);
    w.rec_slot = dalloc<uint32_t>(w.allocs, c);
    w.cap_segs = c;
  }
}

void Matcher::tic(int k) {
  if (!((timing_mask_ >> k) & 1u)) return;
  Ev ev;
  if (!free_ev_.empty()) { ev = free_ev_.back(); free_ev_.pop_back(); }
  else { RM_HIP(hipEventCreate(&ev.a)); RM_HIP(hipEventCreate(&ev.b)); }
  ev.k = k;
  RM_HIP(hipEventRecord(ev.a, stream_));
  pending_.push_back(ev);
}
void Matcher::toc(int k) {
  if (!((timing_mask_ >> k) & 1u) || pending_.empty()) return;
  RM_HIP(hipEventRecord(pending_.back().b, stream_));
}
void Matcher::harvest_times() {
  for (auto& ev : pending_) {
    float ms = 0.f;
    RM_HIP(hipEventElapsedTime(&ms, ev.a, ev.b));
    kms_[ev.k] += ms;
    klaunch_[ev.k] += 1;
    free_ev_.push_back(ev);
  }
  pending_.clear();
}
void Matcher::kernel_times(double* ms, uint64_t* launches) {
  for (int i = 0; i < kNumKernels; ++i) { ms[i] = kms_[i]; if (launches) launches[i] = klaunch_[i]; }
}
void Matcher::reset_kernel_times() {
  for (int i = 0; i < kNumKernels; ++i) { kms_[i] = 0; klaunch_[i] = 0; }
}

void Matcher::sync() {
  RM_HIP(hipStreamSynchronize(stream_));
  harvest_times();
}

// delta-stepping width of the wave search tiers (SearchTargets); RM_SEARCH_DELTA_M overrides
// (0 or negative: plain synchronous rounds)
#ifndef RM_SEARCH_DELTA_M
#define RM_SEARCH_DELTA_M 0
#endif
uint32_t search_delta_cm() {
  static const uint32_t d = [] {
    const char* e = std::getenv("RM_SEARCH_DELTA_M");
    const double m = e && *e ? std::strtod(e, nullptr) : (double)RM_SEARCH_DELTA_M;
    return m > 0.0 ? (uint32_t)std::min(m * 100.0, 4.0e9) : kNone;
  }();
  return d;
}

static DevBatch make_view(const Workspace& w, const InputView& in, uint32_t T, uint64_t P) {
  DevBatch v;
  v.T = T; v.P = P;
  v.trace_off = in.trace_off; v.lon = in.lon; v.lat = in.lat; v.time = in.time; v.acc = in.acc;
  v.opts = in.opts; v.trace_opt = in.trace_opt;
  v.slot_trace = w.slot_trace; v.n_states = w.n_states; v.state_orig = w.state_orig; v.state_time = w.state_time;
  v.cand_n = w.cand_n; v.cand_desc = w.cand_desc; v.cand_sq = w.cand_sq;
  v.trans_cnt = w.trans_cnt; v.trans_off = w.trans_off; v.gc = w.gc; v.route = w.route; v.pair_info = w.pair_info;
  v.route_d = nullptr;   // run_device sets it (and walk) for a batch with turn costs
  v.walk = nullptr;
  v.src_cnt = w.src_cnt; v.src_off = w.src_off; v.src_item = w.src_item;
  v.choice = w.choice; v.chain_start = w.chain_start; v.bp = w.bp;
  v.path_off = w.path_off; v.path_cnt = w.path_cnt; v.path_inline = w.path_inline;
  v.path_pool = w.path_pool; v.path_cap = w.cap_path;
  v.route_dist = w.route_dist; v.path_sab = w.path_sab;
  v.segs = w.segs; v.seg_base = w.seg_base; v.seg_cnt = w.seg_cnt;
  v.trav_off = w.trav_off;
  v.reps = w.reps; v.rep_cnt = w.rep_cnt; v.stats = w.stats;
  v.ctl = w.ctl; v.rl_routes_a = w.rl_routes_a; v.rl_routes_b = w.rl_routes_b; v.rl_routes_0 = w.rl_routes_0;
  v.rl_paths_a = w.rl_paths_a; v.rl_paths_b = w.rl_paths_b; v.rl_cand = w.rl_cand;
  v.rl_routes_c = w.rl_routes_c; v.rl_paths_c = w.rl_paths_c; v.trace_err = w.trace_err;
  v.perm = nullptr;   // run_device sets it when the locality order is on
  v.perm_paths = nullptr;
  v.search_delta = search_delta_cm();
  v.tot = w.tot64;
  v.seg_cap = w.cap_segs;
  v.trans_cap = ~0ull; v.src_cap = ~0ull;
  v.gate = 0;
  return v;
}

// a batch's layout and options, checked before anything is uploaded; sets mode_mask_
void Matcher::check_batch(uint32_t T, const uint32_t* trace_off, const MatchOptions* opts, uint32_t n_opts,
                          const uint32_t* trace_opt) {
  const uint64_t P = trace_off[T];
  if (P >= 0xffffffffull) throw BatchTooLarge("batch too large (points >= 2^32)");
  for (uint32_t k = 0; k < T; ++k) {
    if (trace_off[k + 1] < trace_off[k]) throw std::runtime_error("trace offsets not monotone");
    if (trace_opt[k] >= n_opts) throw std::runtime_error("trace option index out of range");
  }
  scan_options(opts, n_opts);
}

// a batch's option sets, checked; sets mode_mask_, turn_mask_ and batch_radius_
void Matcher::scan_options(const MatchOptions* opts, uint32_t n_opts) {
  mode_mask_ = 0;
  turn_mask_ = 0;
  batch_radius_ = 0.f;
  for (uint32_t q = 0; q < n_opts; ++q) {
    if (opts[q].search_radius > batch_radius_) batch_radius_ = std::min(opts[q].search_radius, kMaxSearchRadius);
    if (opts[q].mode < 0 || opts[q].mode > kModePedestrian) throw std::runtime_error("unknown travel mode");
    // K3 divides by both (a zero 1/beta would turn an invalid route's +inf into NaN)
    if (!(opts[q].sigma_z > 0.f) || !std::isfinite(opts[q].sigma_z)) throw std::runtime_error("sigma_z must be positive and finite");
    if (!(opts[q].beta > 0.f) || !std::isfinite(opts[q].beta)) throw std::runtime_error("beta must be positive and finite");
    if (!turn_factor_ok(opts[q].turn_penalty_factor)) throw std::runtime_error(kTurnPenaltyError);
    mode_mask_ |= 1u << opts[q].mode;
    if (opts[q].turn_penalty_factor > 0.f) turn_mask_ |= 1u << opts[q].mode;
  }
}

// batches of at most this many points take run_small (RM_SMALL_BATCH_POINTS; 0: never)
static uint64_t small_batch_points() {
  const char* e = std::getenv("RM_SMALL_BATCH_POINTS");
  return e && *e ? std::strtoull(e, nullptr, 10) : 65536ull;
}

void Matcher::use_ws_inputs() {
  in_.trace_off = ws_.trace_off; in_.lon = ws_.lon; in_.lat = ws_.lat; in_.time = ws_.time; in_.acc = ws_.acc;
  in_.opts = ws_.opts; in_.trace_opt = ws_.trace_opt;
}

void Matcher::ensure_pack(uint64_t bytes) {
  if (bytes <= pack_cap_ && hpack_ && dpack_) return;
  RM_HIP(hipStreamSynchronize(stream_));   // the previous upload has left the staging
  if (hpack_) (void)hipHostFree(hpack_);
  if (dpack_) (void)hipFree(dpack_);
  hpack_ = nullptr; dpack_ = nullptr; pack_cap_ = 0;
  const uint64_t c = std::max<uint64_t>(bytes + bytes / 2, 1u << 20);
  RM_HIP(hipHostMalloc((void**)&hpack_, c, hipHostMallocDefault));
  std::vector<void*> one;
  grow_workspace([&] { dpack_ = dalloc<char>(one, c); });
  pack_cap_ = c;
}

void Matcher::run(const HostBatch& hb, const RunParams& rp) {
  RM_HIP(hipSetDevice(eng_->device()));
  const uint32_t T = hb.n_traces;
  if (T == 0) { n_traces_ = 0; n_points_ = 0; n_trans_ = 0; n_path_ = 0; seg_used_ = 0; return; }
  const uint64_t P = hb.trace_off[T];
  check_batch(T, hb.trace_off, hb.opts, hb.n_opts, hb.trace_opt);
  {
    // mean sampling interval of the batch: traces sampled sparsely (C3's 30 s) have no spatial
    // coherence from one point to the next, so the locality order pays even on small graphs;
    // at 1 Hz consecutive points share their tables and records already (auto mode)
    double span = 0.0;
    uint64_t gaps = 0;
    for (uint32_t k = 0; k < T; ++k) {
      const uint32_t a = hb.trace_off[k], e = hb.trace_off[k + 1];
      if (e > a + 1) { span += hb.time[e - 1] - hb.time[a]; gaps += e - a - 1; }
    }
    batch_sparse_ = gaps && span / (double)gaps >= kLocalitySparseS;
  }
  ensure(P, T, hb.n_opts);
  Workspace& w = ws_;
  hipStream_t st = stream_;
  if (P <= small_batch_points()) {
    // a small batch goes up as one block through pinned staging: one DMA instead of seven
    // copies (three of them from pageable memory), ~4 us of stream time each
    auto al = [](uint64_t x) { return (x + 15u) & ~(uint64_t)15u; };
    const uint64_t o_topt = (T + 1) * 4ull, o_opts = al(o_topt + T * 4ull);
    const uint64_t o_lon = al(o_opts + hb.n_opts * sizeof(MatchOptions)), o_lat = al(o_lon + P * 4);
    const uint64_t o_acc = al(o_lat + P * 4), o_time = al(o_acc + P * 4), bytes = o_time + P * 8;
    ensure_pack(bytes);
    std::memcpy(hpack_, hb.trace_off, (T + 1) * 4ull);
    std::memcpy(hpack_ + o_topt, hb.trace_opt, T * 4ull);
    std::memcpy(hpack_ + o_opts, hb.opts, hb.n_opts * sizeof(MatchOptions));
    std::memcpy(hpack_ + o_lon, hb.lon, P * 4);
    std::memcpy(hpack_ + o_lat, hb.lat, P * 4);
    std::memcpy(hpack_ + o_acc, hb.accuracy, P * 4);
    std::memcpy(hpack_ + o_time, hb.time, P * 8);
    RM_HIP(hipMemcpyAsync(dpack_, hpack_, bytes, hipMemcpyHostToDevice, st));
    in_.trace_off = (const uint32_t*)dpack_;
    in_.trace_opt = (const uint32_t*)(dpack_ + o_topt);
    in_.opts = (const MatchOptions*)(dpack_ + o_opts);
    in_.lon = (const float*)(dpack_ + o_lon);
    in_.lat = (const float*)(dpack_ + o_lat);
    in_.acc = (const float*)(dpack_ + o_acc);
    in_.time = (const double*)(dpack_ + o_time);
  } else {
    use_ws_inputs();
    RM_HIP(hipMemcpyAsync(w.trace_off, hb.trace_off, (T + 1) * 4ull, hipMemcpyHostToDevice, st));
    RM_HIP(hipMemcpyAsync(w.lon, hb.lon, P * 4, hipMemcpyHostToDevice, st));
    RM_HIP(hipMemcpyAsync(w.lat, hb.lat, P * 4, hipMemcpyHostToDevice, st));
    RM_HIP(hipMemcpyAsync(w.time, hb.time, P * 8, hipMemcpyHostToDevice, st));
    RM_HIP(hipMemcpyAsync(w.acc, hb.accuracy, P * 4, hipMemcpyHostToDevice, st));
    RM_HIP(hipMemcpyAsync(w.opts, hb.opts, hb.n_opts * sizeof(MatchOptions), hipMemcpyHostToDevice, st));
    RM_HIP(hipMemcpyAsync(w.trace_opt, hb.trace_opt, T * 4ull, hipMemcpyHostToDevice, st));
  }
  n_traces_ = T;
  n_points_ = P;
  run_device(rp);
}

// ------------------------------------------------------------------------------------------
// Device JSON parser (rm_match_batch, round 4; DESIGN.md "JSON boundary").  The host reads each
// request's structure (trace_json.hpp parse_request_deferred) and hands over the bytes between
// its trace array's '[' and ']'; here one wave per trace finds the points by their '{' and reads
// them in point_compact's layout only: the keys lat, lon, time, accuracy once each, numbers of at
// most 15 digits without exponent (the values Clinger's exact path gives on the host: one IEEE
// division of two exact doubles), points separated by single commas, lat/lon in range.  Any other
// byte flags the trace and the host parses that request again with the generic reader, so what a
// request returns or fails with never depends on which parser read it.
// The point rules are json_points.hpp's (shared with the host test).
// A wave takes its span 4 KB at a time: the window (and the bytes the points starting in it can
// reach) is copied to LDS with 16-byte loads; 64 ballots over consecutive 64-byte chunks list the
// window's '{' positions in order (consecutive lanes read consecutive bytes: no bank conflicts),
// and lane j reads the window's point j from LDS.
constexpr uint32_t kJsonWin = 4096;     // bytes of span per window
constexpr uint32_t kJsonReach = 256;    // bytes a point may reach past its window (a compact point is < 120)
constexpr uint32_t kJsonLds = kJsonWin + kJsonReach + 16;
constexpr uint64_t kJsonPad = kJsonLds + 64;   // readable bytes the buffer keeps past its last span
constexpr uint32_t kJsonMaxStarts = 128;       // '{' per window (a compact point is >= 40 bytes: <= 103)

__global__ void __launch_bounds__(64) k_parse_json(const uint8_t* s, const uint64_t* span, const uint32_t* trace_off,
                                                   uint32_t T, float* lon, float* lat, double* time, float* acc,
                                                   uint32_t* flag, double2* tspan) {
  __shared__ uint4 win4[kJsonLds / 16];
  __shared__ uint16_t starts[kJsonMaxStarts];
  const uint8_t* win = reinterpret_cast<const uint8_t*>(win4);
  const int lane = threadIdx.x;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (uint32_t k = blockIdx.x; k < T; k += gridDim.x) {
    const uint64_t b = span[2 * k], e = span[2 * k + 1];   // [begin, end) in the byte buffer
    if (b == e) continue;   // parsed on the host
    const uint32_t o = trace_off[k], n = trace_off[k + 1] - o;
    bool bad = false;
    uint32_t base = 0;
    for (uint64_t w = b; w < e; w += kJsonWin) {
      // window bytes [wa, wa + kJsonLds) -> LDS (the buffer is padded: kJsonPad)
      const uint64_t wa = w & ~(uint64_t)15;
      __syncthreads();
      for (uint32_t x = lane; x < kJsonLds / 16; x += 64) win4[x] = reinterpret_cast<const uint4*>(s + wa)[x];
      __syncthreads();
      // positions relative to wa; the loaded bytes end at kJsonLds, the span at er (when inside)
      const uint32_t er = e - wa < (uint64_t)kJsonLds ? (uint32_t)(e - wa) : kJsonLds;
      const bool span_ends = e - wa <= (uint64_t)kJsonLds;
      const uint32_t w0 = (uint32_t)(w - wa), w1 = min(w0 + kJsonWin, er);
      uint32_t ns = 0;
      for (uint32_t c0 = w0; c0 < w1; c0 += 64) {
        const uint32_t pos = c0 + lane;
        const bool open = pos < w1 && win[pos] == '{';
        const unsigned long long m = __ballot(open);
        const uint32_t at = ns + (uint32_t)__popcll(m & below);
        if (open && at < kJsonMaxStarts) starts[at] = (uint16_t)pos;
        ns += (uint32_t)__popcll(m);
      }
      if (ns > kJsonMaxStarts) { bad = true; break; }
      __syncthreads();
      for (uint32_t j = lane; j < ns; j += 64) {
        uint64_t q = starts[j];
        const uint32_t idx = base + j;
        double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
        // a point ending where the loaded bytes end (but not the span) is not read here: flagged
        if (!jp::point(win, q, er, v0, v1, v2, v3) || !jp::point_follows(win, q, er) || (q == er && !span_ends) ||
            !jp::in_range(v0, v1) || idx >= n) {
          bad = true;
          break;
        }
        lat[o + idx] = (float)v0;
        lon[o + idx] = (float)v1;
        time[o + idx] = v2;
        acc[o + idx] = (float)v3;
        if (idx == 0) tspan[k].x = v2;       // the trace's first and last times (the batch's
        if (idx == n - 1) tspan[k].y = v2;   // mean sampling interval, Matcher::run_parsed)
      }
      base += ns;
    }
    if (base != n) bad = true;
    const bool any_bad = __ballot(bad) != 0ull;
    if (lane == 0) flag[k] = any_bad ? 1u : 0u;
  }
}

void Matcher::json_reserve_bytes(uint64_t bytes) {
  RM_HIP(hipSetDevice(eng_->device()));
  if (bytes <= jcap_ && jdev_) return;
  if (jdev_) { RM_HIP(hipStreamSynchronize(stream_)); (void)hipFree(jdev_); jdev_ = nullptr; jcap_ = 0; }
  const uint64_t c = std::max<uint64_t>(bytes + bytes / 4, 1u << 20);
  grow_workspace([&] {
    const hipError_t e = hipMalloc((void**)&jdev_, c + kJsonPad);   // windows read up to kJsonPad past a span
    if (e == hipErrorOutOfMemory) { (void)hipGetLastError(); jdev_ = nullptr; throw OutOfDeviceMemory("JSON buffer"); }
    RM_HIP(e);
  });
  jcap_ = c;
}

void Matcher::json_reserve(uint64_t points, uint32_t traces, uint32_t nopts) {
  RM_HIP(hipSetDevice(eng_->device()));
  ensure(points, traces, nopts);
  if (traces > jtcap_ || !jspan_ || !jflag_ || !jtsp_) {
    RM_HIP(hipStreamSynchronize(stream_));
    for (void* q : {jspan_, (void*)jflag_, jtsp_})
      if (q) (void)hipFree(q);
    jspan_ = nullptr; jflag_ = nullptr; jtsp_ = nullptr;
    jtcap_ = 0;   // a failed allocation below leaves nothing recorded
    const uint32_t c = std::max<uint32_t>(traces + traces / 4 + 1u, 1024u);
    RM_HIP(hipMalloc((void**)&jspan_, (uint64_t)c * 16u));
    RM_HIP(hipMalloc((void**)&jflag_, (uint64_t)c * 4u));
    RM_HIP(hipMalloc((void**)&jtsp_, (uint64_t)c * 16u));
    jtcap_ = c;
  }
}

// thread-safe: the pool threads of rm_match_batch send their arenas as soon as they are filled
void Matcher::json_upload(uint64_t off, const void* src, uint64_t n) {
  if (!n) return;
  if (off + n > jcap_) throw std::runtime_error("json_upload past the reserved buffer");
  RM_HIP(hipSetDevice(eng_->device()));
  RM_HIP(hipMemcpyAsync(jdev_ + off, src, n, hipMemcpyHostToDevice, stream_));
}

void Matcher::json_parse(const uint64_t* span, const uint32_t* trace_off, uint32_t T, uint32_t* flags, double* tspan) {
  if (T > jtcap_ || (uint64_t)trace_off[T] > ws_.cap_points) throw std::runtime_error("json_parse without json_reserve");
  for (uint32_t k = 0; k < T; ++k)
    if (span[2 * k + 1] < span[2 * k] || span[2 * k + 1] > jcap_) throw std::runtime_error("json_parse: span outside the buffer");
  Workspace& w = ws_;
  RM_HIP(hipMemcpyAsync(jspan_, span, T * 16ull, hipMemcpyHostToDevice, stream_));
  RM_HIP(hipMemcpyAsync(w.trace_off, trace_off, (T + 1ull) * 4u, hipMemcpyHostToDevice, stream_));
  RM_HIP(hipMemsetAsync(jflag_, 0, T * 4ull, stream_));
  hipLaunchKernelGGL(k_parse_json, dim3(std::min<uint32_t>(T, 16384u)), dim3(64), 0, stream_, (const uint8_t*)jdev_,
                     (const uint64_t*)jspan_, (const uint32_t*)w.trace_off, T, w.lon, w.lat, w.time, w.acc, jflag_,
                     (double2*)jtsp_);
  RM_HIP(hipGetLastError());
  RM_HIP(hipMemcpyAsync(flags, jflag_, T * 4ull, hipMemcpyDeviceToHost, stream_));
  RM_HIP(hipMemcpyAsync(tspan, jtsp_, T * 16ull, hipMemcpyDeviceToHost, stream_));
  RM_HIP(hipStreamSynchronize(stream_));
}

void Matcher::upload_points(uint64_t first, uint64_t n, const float* lon, const float* lat, const double* time,
                            const float* acc) {
  if (!n) return;
  if (first + n > ws_.cap_points) throw std::runtime_error("upload_points past the reserved points");
  Workspace& w = ws_;
  RM_HIP(hipMemcpyAsync(w.lon + first, lon, n * 4, hipMemcpyHostToDevice, stream_));
  RM_HIP(hipMemcpyAsync(w.lat + first, lat, n * 4, hipMemcpyHostToDevice, stream_));
  RM_HIP(hipMemcpyAsync(w.time + first, time, n * 8, hipMemcpyHostToDevice, stream_));
  RM_HIP(hipMemcpyAsync(w.acc + first, acc, n * 4, hipMemcpyHostToDevice, stream_));
}

void Matcher::run_parsed(const uint32_t* trace_off, uint32_t T, const MatchOptions* opts, uint32_t n_opts,
                         const uint32_t* trace_opt, const double* tspan, const RunParams& rp) {
  RM_HIP(hipSetDevice(eng_->device()));
  if (T == 0) { n_traces_ = 0; n_points_ = 0; n_trans_ = 0; n_path_ = 0; seg_used_ = 0; return; }
  check_batch(T, trace_off, opts, n_opts, trace_opt);
  const uint64_t P = trace_off[T];
  double span = 0.0;
  uint64_t gaps = 0;
  for (uint32_t k = 0; k < T; ++k) {
    const uint32_t a = trace_off[k], e = trace_off[k + 1];
    if (e > a + 1) { span += tspan[2 * k + 1] - tspan[2 * k]; gaps += e - a - 1; }
  }
  batch_sparse_ = gaps && span / (double)gaps >= kLocalitySparseS;
  ensure(P, T, n_opts);   // reserved by json_reserve: no reallocation here (the points are in place)
  use_ws_inputs();
  Workspace& w = ws_;
  hipStream_t st = stream_;
  RM_HIP(hipMemcpyAsync(w.trace_off, trace_off, (T + 1) * 4ull, hipMemcpyHostToDevice, st));
  RM_HIP(hipMemcpyAsync(w.opts, opts, n_opts * sizeof(MatchOptions), hipMemcpyHostToDevice, st));
  RM_HIP(hipMemcpyAsync(w.trace_opt, trace_opt, T * 4ull, hipMemcpyHostToDevice, st));
  n_traces_ = T;
  n_points_ = P;
  run_device(rp);
}

// global-memory search scratch (kGlobalGrid blocks), allocated the first time a search
// outgrows the LDS wave tier
void Matcher::ensure_global_search() {
  if (ws_.gsearch) return;
  ws_.gsearch = dalloc<char>(ws_.allocs, (uint64_t)kGlobalGrid * sizeof(GlobalPathSmem));
}

// read the control words (and nothing else) into hctl_[0..kCtlWords)
void Matcher::read_ctl() {
  RM_HIP(hipMemcpyAsync(hctl_, ws_.ctl, kCtlWords * sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
  RM_HIP(hipStreamSynchronize(stream_));
}

const char* error_text(uint32_t bits) {
  if (bits & kErrCandOverflow) return "too many candidate roads inside the search radius (limit 192)";
  if (bits & kErrSearchOverflow) return "route search exceeded its label capacity (bound too large for this graph)";
  if (bits & kErrRounds) return "route search did not converge / path reconstruction failed";
  return "";
}

// limits of the u32 layouts: route / record offsets are u32 and the record scans take int counts
// that the workspace pads by 1/4 (ensure_segs), so totals must stay below INT32_MAX / 1.25
constexpr uint64_t kMaxTransitions = 0xF0000000ull;
constexpr uint64_t kMaxRecords = 1700000000ull;

// the search tiers' grids (grid-stride over lists the host does not read) shrink with the batch:
// a coalesced service batch of ~15 k points launches them mostly empty
static uint32_t tier_grid(uint64_t P, uint32_t full) {
  return (uint32_t)std::max<uint64_t>(32u, std::min<uint64_t>(full, P / 64u));
}

// Small batches (the coalesced service: a few to a few thousand requests per run).  Their cost
// is latency, not bandwidth: ~45 launches of a few microseconds each, seven uploads and four
// host round trips around ~0.1 ms of kernel work.  Here every pool is sized from upper bounds
// instead of read-back totals (kMaxCand^2 transitions and kMaxCand sources per pair; kInlinePath
// edges per slot in line plus the path pool), the launches that depend on those totals read
// them from the device (DevBatch::tot), the scans fold their partials in one pass, and the
// segment offsets and the compacted reply are prepared before the run's only read-back.  What
// an upper bound cannot cover -- the path pool overflowing, a search handed to the global tier
// before its scratch exists -- gates K4 and the report off on the device (small_abort) and
// returns false: the caller then runs the batch the ordinary way.  Same kernels, same results.
// small runs up to this many points take K1 a wave per state (latency: a lone 1,000-point trace
// 35 -> 10 us; throughput: the lane tier, C2 0.84 ms against 6.45 ms all in the wave tier)
constexpr uint64_t kSmallWaveK1 = 4096;

static ReportArgs report_args(const RunParams& rp) {
  ReportArgs a;
  a.threshold = rp.threshold_sec; a.rmask = rp.report_mask; a.tmask = rp.transition_mask;
  a.hist = rp.hist; a.dur = rp.dur; a.on = rp.do_report ? 1 : 0;
  return a;
}

void Matcher::zero_hist(const RunParams& rp) {
  if (rp.hist) RM_HIP(hipMemsetAsync(rp.hist, 0, (size_t)eng_->n_segments() * kHistBins * sizeof(uint32_t), stream_));
  if (rp.dur) RM_HIP(hipMemsetAsync(rp.dur, 0, (size_t)eng_->n_segments() * 8u, stream_));
}
bool Matcher::run_small(const RunParams& rp, const DevGraph& g) {
  const uint32_t T = n_traces_;
  const uint64_t P = n_points_;
  Workspace& w = ws_;
  hipStream_t st = stream_;
  unsigned long long* htot = reinterpret_cast<unsigned long long*>(hctl_ + 16);
  // sized for the next power of two of points (>= 4,096): a service's batch sizes wander, and each
  // regrowth frees and reallocates (hipFree synchronises the device: a stall of milliseconds)
  uint64_t Pc = 4096;
  while (Pc < P) Pc <<= 1;
  ensure_trans(Pc * kMaxCand * kMaxCand, Pc * kMaxCand);
  if (turn_mask_) ensure_turns();
  ensure_segs(Pc * kInlinePath + w.cap_path);
  DevBatch v = make_view(w, in_, T, P);
  v.route = w.route;
  if (turn_mask_) { v.route_d = w.route_d; v.walk = w.walk; }
  v.src_item = w.src_item;
  v.rl_routes_a = w.rl_routes_a; v.rl_routes_b = w.rl_routes_b; v.rl_routes_0 = w.rl_routes_0;
  v.rl_routes_c = w.rl_routes_c;
  v.segs = w.segs; v.reps = w.reps; v.seg_cap = w.cap_segs;
  v.gate = w.gsearch ? 1u : 3u;
  locality_used_ = false;   // a few thousand points: nothing to gain from the region order
  const uint32_t count_grid = (uint32_t)((P + 255) / 256);
  const uint32_t sum_grid = (uint32_t)((P + 1023) / 1024);
  const uint64_t max_src = P * kMaxCand;
  const uint32_t item_grid = (uint32_t)((max_src + kK2Items - 1) / kK2Items);
  const uint32_t lane_grid = (uint32_t)((max_src + 255) / 256);
  const auto tgrid = [P](uint32_t full) { return tier_grid(P, full); };

  tic(kKStates);
  hipLaunchKernelGGL(k_states, dim3(T), dim3(64), 0, st, v);
  toc(kKStates);
  tic(kKCandidates);
  DevGraph gk = g;   // K1's grid for the batch's radius
  eng_->k1_grid(batch_radius_, gk);
  if (P <= kSmallWaveK1) {   // one wave per state
    hipLaunchKernelGGL(k_candidates_wave, dim3((uint32_t)P), dim3(64), 0, st, gk, v, 1);
  } else {
    hipLaunchKernelGGL(k_candidates_lane, dim3(count_grid), dim3(256), 0, st, gk, v);
    hipLaunchKernelGGL(k_candidates_wave, dim3(tgrid(2048)), dim3(64), 0, st, gk, v, 0);
  }
  toc(kKCandidates);
  tic(kKScan);
  hipLaunchKernelGGL(k_trans_count, dim3(count_grid), dim3(256), 0, st, v, w.tot_part);
  hipLaunchKernelGGL(k_trans_apply_small, dim3(count_grid), dim3(256), 0, st, v, (const unsigned long long*)w.tot_part,
                     count_grid, w.tot64);
  toc(kKScan);
  const bool balls = (mode_mask_ & g.ball_mask) != 0u;
  // the short hand-over chain (k_routes_grp): with the route tables most small batches hand over
  // nothing, and the five-tier chain's launches were a sixth of their engine time;
  // RM_SMALL_SHORT_CHAIN=0 launches every tier (A/B)
  const char* sc_env = std::getenv("RM_SMALL_SHORT_CHAIN");   // (read per run: tests switch it)
  const bool short_chain = balls && !(sc_env && *sc_env == '0');
  tic(kKRoutes);
  if (balls) {
    if (v.route_d) {
      hipLaunchKernelGGL(k_routes_ball2<true>, dim3(item_grid), dim3(kK2Threads), 0, st, g, v, kNone);
      hipLaunchKernelGGL(k_turn_walks, dim3(item_grid), dim3(kWalkThreads), 0, st, g, v, kNone);
      hipLaunchKernelGGL(k_turn_walks_marked, dim3(kWalkScanGrid), dim3(256), 0, st, g, v);
    } else {
      hipLaunchKernelGGL(k_routes_ball2<false>, dim3(item_grid), dim3(kK2Threads), 0, st, g, v, kNone);
    }
    if (!short_chain) {
      const uint32_t lg = (uint32_t)std::min<uint64_t>(lane_grid, kListedGrid);
      if (v.route_d) hipLaunchKernelGGL(k_routes_lane<true>, dim3(lg), dim3(256), 0, st, g, v, 0u, 1);
      else hipLaunchKernelGGL(k_routes_lane<false>, dim3(lg), dim3(256), 0, st, g, v, 0u, 1);
    }
  } else {
    if (v.route_d) hipLaunchKernelGGL(k_routes_lane<true>, dim3(lane_grid), dim3(256), 0, st, g, v, kNone, 0);
    else hipLaunchKernelGGL(k_routes_lane<false>, dim3(lane_grid), dim3(256), 0, st, g, v, kNone, 0);
  }
  if (!short_chain) hipLaunchKernelGGL(k_routes_reg2, dim3(tgrid(kReg2Grid)), dim3(256), 0, st, g, v);
  hipLaunchKernelGGL(k_routes_grp, dim3(tgrid(kGrpGrid)), dim3(64), 0, st, g, v, short_chain ? 1 : 0);
  if (!short_chain) hipLaunchKernelGGL(k_routes_wave_s, dim3(tgrid(kMidGrid)), dim3(64), 0, st, g, v);
  hipLaunchKernelGGL(k_routes_wave, dim3(tgrid(1024)), dim3(64), 0, st, g, v, short_chain ? 1 : 0);
  if (w.gsearch) hipLaunchKernelGGL(k_routes_global, dim3(kGlobalGrid), dim3(64), 0, st, g, v, (GlobalPathSmem*)w.gsearch);
  toc(kKRoutes);
  tic(kKViterbi);
  launch_viterbi(T, st, v);
  toc(kKViterbi);
  tic(kKPaths);
  if (balls) {
    hipLaunchKernelGGL(k_paths_ball, dim3(count_grid), dim3(256), 0, st, g, v);
    if (!short_chain)
      hipLaunchKernelGGL(k_paths_lane, dim3((uint32_t)std::min<uint64_t>(count_grid, kListedGrid)), dim3(256), 0, st, g, v, 1);
  } else {
    hipLaunchKernelGGL(k_paths_lane, dim3(count_grid), dim3(256), 0, st, g, v, 0);
  }
  if (!short_chain) hipLaunchKernelGGL(k_paths_reg2, dim3(tgrid(kReg2Grid)), dim3(256), 0, st, g, v);
  hipLaunchKernelGGL(k_paths_grp, dim3(tgrid(kGrpGrid)), dim3(64), 0, st, g, v, short_chain ? 1 : 0);
  if (!short_chain) hipLaunchKernelGGL(k_paths_wave_s, dim3(tgrid(kMidGrid)), dim3(64), 0, st, g, v);
  hipLaunchKernelGGL(k_paths_wave, dim3(tgrid(1024)), dim3(64), 0, st, g, v, short_chain ? 1 : 0);
  if (w.gsearch) hipLaunchKernelGGL(k_paths_global, dim3(kGlobalGrid), dim3(64), 0, st, g, v, (GlobalPathSmem*)w.gsearch);
  toc(kKPaths);
  tic(kKSegments);
  hipLaunchKernelGGL(k_sum_u64, dim3(sum_grid), dim3(256), 0, st, w.path_cnt, P, w.tot_part);
  hipLaunchKernelGGL(k_path_apply_small, dim3(sum_grid), dim3(256), 0, st, v, (const unsigned long long*)w.tot_part,
                     sum_grid, w.tot64, w.rec_slot);
  if (rp.do_report && rp.zero_hist) zero_hist(rp);
  hipLaunchKernelGGL(k_seg_wave, dim3(T), dim3(64), 0, st, g, v, (const uint32_t*)w.rec_slot, kNone, report_args(rp));
  toc(kKSegments);
  // the reply's segments, compacted per trace on the device (get_segments then copies them down)
  constexpr uint32_t kSegWords = sizeof(SegmentRec) / 8;
  const size_t offb = ((T + 1) * 4ull + 7) & ~(size_t)7;
  bool prefetch = rp.prefetch_segments != 0;
  if (prefetch) {
    try {
      grow_dl_dev(offb + v.seg_cap * sizeof(SegmentRec));
    } catch (const BatchTooLarge&) {
      prefetch = false;   // the ordinary download sizes its buffer from the counts instead
    }
  }
  if (prefetch) {
    if (T + 1 > hoff_cap_) {
      if (hoff_) RM_HIP(hipHostFree(hoff_));
      hoff_ = nullptr; hoff_cap_ = 0;
      const uint64_t c = std::max<uint64_t>(T + 1 + T / 2, 4096);
      RM_HIP(hipHostMalloc((void**)&hoff_, c * 4, hipHostMallocDefault));
      hoff_cap_ = c;
    }
    uint32_t* d_off = (uint32_t*)dl_dev_;
    hipLaunchKernelGGL(k_seg_offsets_small, dim3(1), dim3(1024), 0, st, v, d_off);
    hipLaunchKernelGGL(k_gather_recs, dim3(std::min<uint32_t>(T, 8192u)), dim3(64), 0, st, T, (const uint32_t*)w.seg_base,
                       (const uint32_t*)w.seg_cnt, (const uint32_t*)d_off, (const unsigned long long*)w.segs, kSegWords,
                       (unsigned long long*)((char*)dl_dev_ + offb));
    RM_HIP(hipMemcpyAsync(hoff_, d_off, (T + 1) * 4ull, hipMemcpyDeviceToHost, st));
  }
  RM_HIP(hipGetLastError());
  RM_HIP(hipMemcpyAsync(hctl_, w.ctl, kCtlWords * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  RM_HIP(hipMemcpyAsync(htot, w.tot64, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  sync();
  if ((hctl_[2] & kErrPathOverflow) || (!w.gsearch && (hctl_[9] | hctl_[10])) || htot[2] > v.seg_cap) return false;
  n_trans_ = htot[0];
  n_path_ = htot[2];
  seg_used_ = htot[2];
  has_report_ = rp.do_report != 0;
  seg_prefetched_ = prefetch;
  err_bits_ = hctl_[2] & (kErrCandOverflow | kErrSearchOverflow | kErrRounds);
  if (err_bits_ && !isolate_) throw std::runtime_error(error_text(err_bits_));
  return true;
}

// Large batches in steady state (round 5): the ordinary path reads two totals back in the middle
// of a run -- the transitions and K2 sources after the candidate scan (to size the route pools and
// K2's grid) and the traversal records after the path stage -- two host round trips of ~30 us
// each (5 % of a C2 step's gaps).  A matcher whose previous run left its pools sized runs the
// same kernels without them: K2's grid covers the previous run's sources and an eighth more and
// reads the count on the device, the traversal records and the path-stage hand-overs are checked
// on the device, and a batch that outgrows any of it is gated off after the scan (steady_abort:
// every stage skips it; small_abort for K4 and the report) and run again the ordinary way.  No
// locality order (its permuted K2 item scan stays on the ordinary path).  RM_STEADY=0: off.
bool Matcher::run_steady(const RunParams& rp, const DevGraph& g) {
  const uint32_t T = n_traces_;
  const uint64_t P = n_points_;
  Workspace& w = ws_;
  hipStream_t st = stream_;
  unsigned long long* htot = reinterpret_cast<unsigned long long*>(hctl_ + 16);
  if (turn_mask_) ensure_turns();
  DevBatch v = make_view(w, in_, T, P);
  v.route = w.route;
  if (turn_mask_) { v.route_d = w.route_d; v.walk = w.walk; }
  v.src_item = w.src_item;
  v.rl_routes_a = w.rl_routes_a; v.rl_routes_b = w.rl_routes_b; v.rl_routes_0 = w.rl_routes_0;
  v.rl_routes_c = w.rl_routes_c;
  v.segs = w.segs; v.reps = w.reps; v.seg_cap = w.cap_segs;
  const uint64_t src_cover = std::min<uint64_t>(w.cap_src, steady_src_ + steady_src_ / 8 + 4096);
  v.trans_cap = w.cap_trans;
  v.src_cap = src_cover;
  v.gate = (w.gsearch ? 1u : 3u) | 4u;
  locality_used_ = false;
  const uint32_t count_grid = (uint32_t)((P + 255) / 256);
  const uint32_t sum_grid = (uint32_t)((P + 1023) / 1024);
  // the hand-over tiers' grids from the previous run's list lengths (each is a grid-stride loop:
  // any grid is correct, and a list that grew runs on fewer blocks than it could): mostly empty
  // launches of 64 blocks instead of up to 4,096
  static const bool prev_grids = [] { const char* e = std::getenv("RM_STEADY_GRIDS"); return !(e && *e == '0'); }();   // A/B
  const auto sgrid = [&](uint32_t full, int word, uint32_t per_block) {
    if (!prev_grids) return (uint32_t)(full == 2048u ? 2048u : tier_grid(P, full));
    const uint64_t want = 4ull * (((uint64_t)steady_ctl_[word] + per_block - 1) / per_block);
    return (uint32_t)std::min<uint64_t>(tier_grid(P, full), std::max<uint64_t>(64u, want));
  };

  tic(kKStates);
  hipLaunchKernelGGL(k_states, dim3(T), dim3(64), 0, st, v);
  toc(kKStates);
  tic(kKCandidates);
  DevGraph gk = g;
  eng_->k1_grid(batch_radius_, gk);
  hipLaunchKernelGGL(k_candidates_lane, dim3(count_grid), dim3(256), 0, st, gk, v);
  hipLaunchKernelGGL(k_candidates_wave, dim3(sgrid(2048, 7, 1)), dim3(64), 0, st, gk, v, 0);
  toc(kKCandidates);
  tic(kKScan);
  hipLaunchKernelGGL(k_trans_count, dim3(count_grid), dim3(256), 0, st, v, w.tot_part);
  hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(1024), 0, st, w.tot_part, count_grid, w.tot64);
  hipLaunchKernelGGL(k_scan_apply2, dim3(count_grid), dim3(256), 0, st, (const uint32_t*)w.trans_cnt,
                     (const uint32_t*)w.src_cnt, P, (const unsigned long long*)w.tot_part, w.trans_off, w.src_off);
  toc(kKScan);
  const bool balls = (mode_mask_ & g.ball_mask) != 0u;
  const uint32_t item_grid = (uint32_t)((src_cover + kK2Items - 1) / kK2Items);
  const uint32_t lane_grid = (uint32_t)((src_cover + 255) / 256);
  tic(kKRoutes);
  hipLaunchKernelGGL(k_src_items, dim3(count_grid), dim3(256), 0, st, v);
  if (balls) {
    if (v.route_d) {
      hipLaunchKernelGGL(k_routes_ball2<true>, dim3(item_grid), dim3(kK2Threads), 0, st, g, v, kNone);
      hipLaunchKernelGGL(k_turn_walks, dim3(item_grid), dim3(kWalkThreads), 0, st, g, v, kNone);
      hipLaunchKernelGGL(k_turn_walks_marked, dim3(kWalkScanGrid), dim3(256), 0, st, g, v);
    } else {
      hipLaunchKernelGGL(k_routes_ball2<false>, dim3(item_grid), dim3(kK2Threads), 0, st, g, v, kNone);
    }
    const uint32_t lg = std::min<uint32_t>(lane_grid, sgrid(kListedGrid, 1, 256));
    if (v.route_d) hipLaunchKernelGGL(k_routes_lane<true>, dim3(lg), dim3(256), 0, st, g, v, 0u, 1);
    else hipLaunchKernelGGL(k_routes_lane<false>, dim3(lg), dim3(256), 0, st, g, v, 0u, 1);
  } else {
    if (v.route_d) hipLaunchKernelGGL(k_routes_lane<true>, dim3(lane_grid), dim3(256), 0, st, g, v, kNone, 0);
    else hipLaunchKernelGGL(k_routes_lane<false>, dim3(lane_grid), dim3(256), 0, st, g, v, kNone, 0);
  }
  hipLaunchKernelGGL(k_routes_reg2, dim3(sgrid(kReg2Grid, 3, 256)), dim3(256), 0, st, g, v);
  hipLaunchKernelGGL(k_routes_grp, dim3(sgrid(kGrpGrid, 5, kWave / kGrpW)), dim3(64), 0, st, g, v, 0);
  hipLaunchKernelGGL(k_routes_wave_s, dim3(sgrid(kMidGrid, 11, 1)), dim3(64), 0, st, g, v);
  hipLaunchKernelGGL(k_routes_wave, dim3(sgrid(1024, 13, 1)), dim3(64), 0, st, g, v, 0);
  if (w.gsearch) hipLaunchKernelGGL(k_routes_global, dim3(kGlobalGrid), dim3(64), 0, st, g, v, (GlobalPathSmem*)w.gsearch);
  toc(kKRoutes);
  tic(kKViterbi);
  launch_viterbi(T, st, v);
  toc(kKViterbi);
  tic(kKPaths);
  if (balls) {
    hipLaunchKernelGGL(k_paths_ball, dim3(count_grid), dim3(256), 0, st, g, v);
    hipLaunchKernelGGL(k_paths_lane, dim3(std::min<uint32_t>(count_grid, sgrid(kListedGrid, 8, 256))), dim3(256), 0, st, g, v, 1);
  } else {
    hipLaunchKernelGGL(k_paths_lane, dim3(count_grid), dim3(256), 0, st, g, v, 0);
  }
  hipLaunchKernelGGL(k_paths_reg2, dim3(sgrid(kReg2Grid, 4, 256)), dim3(256), 0, st, g, v);
  hipLaunchKernelGGL(k_paths_grp, dim3(sgrid(kGrpGrid, 6, kWave / kGrpW)), dim3(64), 0, st, g, v, 0);
  hipLaunchKernelGGL(k_paths_wave_s, dim3(sgrid(kMidGrid, 12, 1)), dim3(64), 0, st, g, v);
  hipLaunchKernelGGL(k_paths_wave, dim3(sgrid(1024, 14, 1)), dim3(64), 0, st, g, v, 0);
  if (w.gsearch) hipLaunchKernelGGL(k_paths_global, dim3(kGlobalGrid), dim3(64), 0, st, g, v, (GlobalPathSmem*)w.gsearch);
  toc(kKPaths);
  tic(kKSegments);
  hipLaunchKernelGGL(k_sum_u64, dim3(sum_grid), dim3(256), 0, st, w.path_cnt, P, w.tot_part);
  hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(1024), 0, st, w.tot_part, sum_grid, w.tot64 + 2);
  hipLaunchKernelGGL(k_scan_apply4, dim3(sum_grid), dim3(256), 0, st, (const uint32_t*)w.path_cnt, P,
                     (const unsigned long long*)w.tot_part, w.trav_off);
  if (rp.do_report && rp.zero_hist) zero_hist(rp);
  hipLaunchKernelGGL(k_rec_slot, dim3(count_grid), dim3(256), 0, st, v, w.rec_slot);
  hipLaunchKernelGGL(k_seg_wave, dim3(T), dim3(64), 0, st, g, v, (const uint32_t*)w.rec_slot, kNone, report_args(rp));
  toc(kKSegments);
  RM_HIP(hipGetLastError());
  RM_HIP(hipMemcpyAsync(hctl_, w.ctl, kCtlWords * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  RM_HIP(hipMemcpyAsync(htot, w.tot64, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  sync();
  if (htot[0] > w.cap_trans || htot[1] > src_cover || (hctl_[2] & kErrPathOverflow) ||
      (!w.gsearch && (hctl_[9] | hctl_[10])) || htot[2] > v.seg_cap)
    return false;
  n_trans_ = htot[0];
  n_path_ = htot[2];
  seg_used_ = htot[2];
  steady_src_ = htot[1];
  std::memcpy(steady_ctl_, hctl_, sizeof(steady_ctl_));
  has_report_ = rp.do_report != 0;
  err_bits_ = hctl_[2] & (kErrCandOverflow | kErrSearchOverflow | kErrRounds);
  if (err_bits_ && !isolate_) throw std::runtime_error(error_text(err_bits_));
  return true;
}

void Matcher::run_device(const RunParams& rp) {
  RM_HIP(hipSetDevice(eng_->device()));
  const uint32_t T = n_traces_;
  const uint64_t P = n_points_;
  err_bits_ = 0;
  if (T == 0) return;
  if (P >= (uint64_t)kTravLast) throw BatchTooLarge("batch too large (slots >= 2^30); split it");  // TravRec::slot flags
  Workspace& w = ws_;
  hipStream_t st = stream_;
  eng_->ensure_balls(mode_mask_);
  if (turn_mask_) eng_->ensure_turn_rows(turn_mask_);
  const DevGraph g = eng_->dev_snapshot();
  if (!hctl_) RM_HIP(hipHostMalloc((void**)&hctl_, 32 * sizeof(uint32_t), hipHostMallocDefault));
  unsigned long long* htot = reinterpret_cast<unsigned long long*>(hctl_ + 16);
  seg_prefetched_ = false;
  // (a forced locality order takes the ordinary path: the small one runs in slot order)
  if (P <= small_batch_points() && locality_ <= 0 && run_small(rp, g)) return;
  const char* steady_env = std::getenv("RM_STEADY");   // (read per run: tests switch it)
  const bool steady_on = !(steady_env && *steady_env == '0');
  if (steady_on && steady_src_ && w.route && w.src_item && w.path_pool && w.segs && T > 0) {
    int lm = locality_;
    if (lm < 0) lm = eng_->locality_default() ? 2 : (batch_sparse_ ? 1 : 0);
    if (eng_->locality_bits() == 0) lm = 0;
    if (lm == 0 && run_steady(rp, g)) return;
    steady_src_ = 0;   // (re-armed by the ordinary run below)
  }
  // (k_states zeroes the control words and the per-trace error bits)
  DevBatch v = make_view(w, in_, T, P);
  const uint32_t count_grid = (uint32_t)((P + 255) / 256);
  const uint32_t sum_grid = (uint32_t)((P + 1023) / 1024);   // k_sum_u64: four counts per lane

  tic(kKStates);
  hipLaunchKernelGGL(k_states, dim3(T), dim3(64), 0, st, v);
  toc(kKStates);
  // mode: 0 slot order, 1 K1 + K2 in locality order, 2 the path stage too; auto (-1): 2 on large
  // graphs, 1 for sparsely sampled batches on small ones (measured: DESIGN.md §5 "Locality")
  int lmode = locality_;
  if (lmode < 0) lmode = eng_->locality_default() ? 2 : (batch_sparse_ ? 1 : 0);
  if (eng_->locality_bits() == 0) lmode = 0;   // one region: nothing to order
  locality_used_ = lmode > 0;
  if (locality_used_) {
    tic(kKLocality);
    ensure_sort(P);
    const uint32_t lgrid = (uint32_t)((P + 256u * kLocPerThread - 1) / (256u * kLocPerThread));
    RM_HIP(hipMemsetAsync(w.loc_cursor, 0, (kLocBuckets + 1) * sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_loc_count, dim3(lgrid), dim3(256), 0, st, g, v, eng_->locality_shift(), w.loc_key,
                       w.loc_cursor);
    hipLaunchKernelGGL(k_loc_scan, dim3(1), dim3(1024), 0, st, w.loc_cursor);
    hipLaunchKernelGGL(k_loc_scatter, dim3(lgrid), dim3(256), 0, st, P, (const uint16_t*)w.loc_key, w.loc_cursor, w.perm);
    v.perm = w.perm;
    if (lmode >= 2) v.perm_paths = w.perm;
    toc(kKLocality);
  }
  tic(kKCandidates);
  DevGraph gk = g;   // K1's grid for the batch's radius
  eng_->k1_grid(batch_radius_, gk);
  static const bool k1_wave_all = [] { const char* e = std::getenv("RM_K1_WAVE_ALL"); return e && *e == '1'; }();
  if (k1_wave_all) {   // A/B: every state in the wave tier
    hipLaunchKernelGGL(k_candidates_wave, dim3((uint32_t)std::min<uint64_t>(P, 1u << 20)), dim3(64), 0, st, gk, v, 1);
  } else {
    hipLaunchKernelGGL(k_candidates_lane, dim3((uint32_t)((P + 255) / 256)), dim3(256), 0, st, gk, v);
    hipLaunchKernelGGL(k_candidates_wave, dim3(2048), dim3(64), 0, st, gk, v, 0);
  }
  toc(kKCandidates);
  tic(kKScan);
  hipLaunchKernelGGL(k_trans_count, dim3(count_grid), dim3(256), 0, st, v, w.tot_part);
  hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(1024), 0, st, w.tot_part, count_grid, w.tot64);
  hipLaunchKernelGGL(k_scan_apply2, dim3(count_grid), dim3(256), 0, st, (const uint32_t*)w.trans_cnt,
                     (const uint32_t*)w.src_cnt, P, (const unsigned long long*)w.tot_part, w.trans_off, w.src_off);
  if (v.perm) {   // K2 items in locality order: src_off from a scan of the counts in perm order
    hipLaunchKernelGGL(k_perm_src_count, dim3(count_grid), dim3(256), 0, st, v, w.pcnt, w.tot_part);
    hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(1024), 0, st, w.tot_part, count_grid, w.tot64 + 2);
    hipLaunchKernelGGL(k_scan_apply_perm, dim3(count_grid), dim3(256), 0, st, (const uint32_t*)w.pcnt, P,
                       (const unsigned long long*)w.tot_part, (const uint32_t*)w.perm, w.src_off);
  }
  toc(kKScan);
  RM_HIP(hipMemcpyAsync(htot, w.tot64, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  RM_HIP(hipStreamSynchronize(st));
  const uint64_t total = htot[0];
  const uint64_t n_src = htot[1];
  if (total >= kMaxTransitions) throw BatchTooLarge("batch too large (transitions >= 0xF0000000); split it");
  uint64_t steady_next = n_src ? n_src : 1;   // a later batch may run steady (run_steady) from these pools
  n_trans_ = total;
  ensure_trans(total, n_src);
  v.route = w.route;
  if (turn_mask_) {   // the transitions' distance terms with turn costs (rule 3b), read by K3
    ensure_turns();
    v.route_d = w.route_d;
    v.walk = w.walk;
  }
  v.src_item = w.src_item;
  v.rl_routes_a = w.rl_routes_a;
  v.rl_routes_b = w.rl_routes_b;
  v.rl_routes_0 = w.rl_routes_0;
  v.rl_routes_c = w.rl_routes_c;

  // the ball tiers run when some mode of the batch has route balls; items of a mode without
  // them (or bounds above its radius) are handed to the search tiers
  const bool balls = (mode_mask_ & g.ball_mask) != 0u;
  tic(kKRoutes);
  hipLaunchKernelGGL(k_src_items, dim3((uint32_t)((P + 255) / 256)), dim3(256), 0, st, v);
  if (n_src && balls) {
    if (v.route_d) {
      hipLaunchKernelGGL(k_routes_ball2<true>, dim3((uint32_t)((n_src + kK2Items - 1) / kK2Items)), dim3(kK2Threads), 0, st,
                         g, v, (uint32_t)n_src);
      hipLaunchKernelGGL(k_turn_walks, dim3((uint32_t)((n_src + kK2Items - 1) / kK2Items)), dim3(kWalkThreads), 0, st, g, v,
                         (uint32_t)n_src);
      hipLaunchKernelGGL(k_turn_walks_marked, dim3(kWalkScanGrid), dim3(256), 0, st, g, v);
    } else
      hipLaunchKernelGGL(k_routes_ball2<false>, dim3((uint32_t)((n_src + kK2Items - 1) / kK2Items)), dim3(kK2Threads), 0, st,
                         g, v, (uint32_t)n_src);
    if (v.route_d)
      hipLaunchKernelGGL(k_routes_lane<true>, dim3((uint32_t)std::min<uint64_t>((n_src + 255) / 256, kListedGrid)), dim3(256),
                         0, st, g, v, 0u, 1);
    else
      hipLaunchKernelGGL(k_routes_lane<false>, dim3((uint32_t)std::min<uint64_t>((n_src + 255) / 256, kListedGrid)),
                         dim3(256), 0, st, g, v, 0u, 1);
  } else if (n_src) {
    if (v.route_d)
      hipLaunchKernelGGL(k_routes_lane<true>, dim3((uint32_t)((n_src + 255) / 256)), dim3(256), 0, st, g, v, (uint32_t)n_src, 0);
    else
      hipLaunchKernelGGL(k_routes_lane<false>, dim3((uint32_t)((n_src + 255) / 256)), dim3(256), 0, st, g, v, (uint32_t)n_src, 0);
  }
  // the search tiers' grids (grid-stride over lists the host does not read) shrink with the batch:
  // a coalesced service batch of ~15 k points launches them mostly empty
  const auto tgrid = [P](uint32_t full) { return tier_grid(P, full); };
  hipLaunchKernelGGL(k_routes_reg2, dim3(tgrid(kReg2Grid)), dim3(256), 0, st, g, v);
  hipLaunchKernelGGL(k_routes_grp, dim3(tgrid(kGrpGrid)), dim3(64), 0, st, g, v, 0);
  hipLaunchKernelGGL(k_routes_wave_s, dim3(tgrid(kMidGrid)), dim3(64), 0, st, g, v);
  hipLaunchKernelGGL(k_routes_wave, dim3(tgrid(1024)), dim3(64), 0, st, g, v, 0);
  // the global tier runs in line once its scratch exists; before that, a hand-over seen at the
  // path-stage read-back allocates it and re-runs K3 (rare: bounds of many kilometres)
  bool routes_global_done = w.gsearch != nullptr;
  if (routes_global_done)
    hipLaunchKernelGGL(k_routes_global, dim3(kGlobalGrid), dim3(64), 0, st, g, v, (GlobalPathSmem*)w.gsearch);
  toc(kKRoutes);
  tic(kKViterbi);
  launch_viterbi(T, st, v);
  toc(kKViterbi);
  for (int attempt = 0;; ++attempt) {
    tic(kKPaths);
    if (attempt) {   // the first attempt starts from the zeroed control words
      RM_HIP(hipMemsetAsync(w.ctl + 8, 0, sizeof(uint32_t), st));    // path ball hand-overs
      RM_HIP(hipMemsetAsync(w.ctl + 10, 0, sizeof(uint32_t), st));   // paths list C
      RM_HIP(hipMemsetAsync(w.ctl + 12, 0, sizeof(uint32_t), st));   // paths list B2
      RM_HIP(hipMemsetAsync(w.ctl + 14, 0, sizeof(uint32_t), st));   // paths list B3
    }
    if (balls) {
      hipLaunchKernelGGL(k_paths_ball, dim3((uint32_t)((P + 255) / 256)), dim3(256), 0, st, g, v);
      hipLaunchKernelGGL(k_paths_lane, dim3((uint32_t)std::min<uint64_t>((P + 255) / 256, kListedGrid)), dim3(256), 0,
                         st, g, v, 1);
    } else {
      hipLaunchKernelGGL(k_paths_lane, dim3((uint32_t)((P + 255) / 256)), dim3(256), 0, st, g, v, 0);
    }
    hipLaunchKernelGGL(k_paths_reg2, dim3(tgrid(kReg2Grid)), dim3(256), 0, st, g, v);
    hipLaunchKernelGGL(k_paths_grp, dim3(tgrid(kGrpGrid)), dim3(64), 0, st, g, v, 0);
    hipLaunchKernelGGL(k_paths_wave_s, dim3(tgrid(kMidGrid)), dim3(64), 0, st, g, v);
    hipLaunchKernelGGL(k_paths_wave, dim3(tgrid(1024)), dim3(64), 0, st, g, v, 0);
    if (w.gsearch) hipLaunchKernelGGL(k_paths_global, dim3(kGlobalGrid), dim3(64), 0, st, g, v, (GlobalPathSmem*)w.gsearch);
    toc(kKPaths);
    // traversal records are laid out by a scan of path_cnt (0 for slots without a chosen transition)
    tic(kKSegments);
    hipLaunchKernelGGL(k_sum_u64, dim3(sum_grid), dim3(256), 0, st, w.path_cnt, P, w.tot_part);
    hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(1024), 0, st, w.tot_part, sum_grid, w.tot64 + 2);
    hipLaunchKernelGGL(k_scan_apply4, dim3(sum_grid), dim3(256), 0, st, (const uint32_t*)w.path_cnt, P,
                       (const unsigned long long*)w.tot_part, w.trav_off);
    toc(kKSegments);
    RM_HIP(hipMemcpyAsync(htot + 2, w.tot64 + 2, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    read_ctl();
    if (!routes_global_done && hctl_[9]) {
      // routes outgrew the LDS wave tier: run them in the global tier, then K3 and paths again
      ensure_global_search();
      routes_global_done = true;
      hipLaunchKernelGGL(k_routes_global, dim3(kGlobalGrid), dim3(64), 0, st, g, v, (GlobalPathSmem*)w.gsearch);
      launch_viterbi(T, st, v);
      RM_HIP(hipMemsetAsync(w.path_cnt, 0, P * sizeof(uint32_t), st));
      for (int c : {0, 4, 6}) RM_HIP(hipMemsetAsync(w.ctl + c, 0, sizeof(uint32_t), st));
      uint32_t flags = hctl_[2] & ~kErrPathOverflow;
      RM_HIP(hipMemcpyAsync(w.ctl + 2, &flags, sizeof(uint32_t), hipMemcpyHostToDevice, st));
      RM_HIP(hipStreamSynchronize(st));
      continue;
    }
    if (!w.gsearch && hctl_[10]) {
      // chosen transitions whose path search outgrew the LDS wave tier
      ensure_global_search();
      hipLaunchKernelGGL(k_paths_global, dim3(kGlobalGrid), dim3(64), 0, st, g, v, (GlobalPathSmem*)w.gsearch);
      hipLaunchKernelGGL(k_sum_u64, dim3(sum_grid), dim3(256), 0, st, w.path_cnt, P, w.tot_part);
      hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(1024), 0, st, w.tot_part, sum_grid, w.tot64 + 2);
      hipLaunchKernelGGL(k_scan_apply4, dim3(sum_grid), dim3(256), 0, st, (const uint32_t*)w.path_cnt, P,
                         (const unsigned long long*)w.tot_part, w.trav_off);
      RM_HIP(hipMemcpyAsync(htot + 2, w.tot64 + 2, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
      read_ctl();
    }
    if (!(hctl_[2] & kErrPathOverflow)) break;
    if (attempt > 3) throw BatchTooLarge("path pool overflow persists");
    ensure_path((uint64_t)hctl_[0]);
    v.path_pool = w.path_pool; v.path_cap = w.cap_path;
    RM_HIP(hipMemsetAsync(w.ctl, 0, sizeof(uint32_t), st));          // path_used
    RM_HIP(hipMemsetAsync(w.ctl + 4, 0, sizeof(uint32_t), st));      // paths list A
    RM_HIP(hipMemsetAsync(w.ctl + 6, 0, sizeof(uint32_t), st));      // paths list B
    uint32_t flags = hctl_[2] & ~kErrPathOverflow;
    RM_HIP(hipMemcpyAsync(w.ctl + 2, &flags, sizeof(uint32_t), hipMemcpyHostToDevice, st));
    RM_HIP(hipStreamSynchronize(st));
  }
  const uint64_t seg_total = htot[2];
  if (seg_total >= kMaxRecords) throw BatchTooLarge("batch too large (path edges >= 1.7e9); split it");
  n_path_ = seg_total;  // one traversal record (and at most one segment) per chosen path edge
  ensure_segs(seg_total);
  v.segs = w.segs; v.reps = w.reps; v.seg_cap = w.cap_segs;
  tic(kKSegments);
  if (rp.do_report && rp.zero_hist) zero_hist(rp);
  if (T) {
    hipLaunchKernelGGL(k_rec_slot, dim3((uint32_t)((P + 255) / 256)), dim3(256), 0, st, v, w.rec_slot);
    hipLaunchKernelGGL(k_seg_wave, dim3(T), dim3(64), 0, st, g, v, (const uint32_t*)w.rec_slot, (uint32_t)seg_total,
                       report_args(rp));
  }
  toc(kKSegments);
  RM_HIP(hipGetLastError());
  RM_HIP(hipMemcpyAsync(hctl_, w.ctl, kCtlWords * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  sync();
  seg_used_ = seg_total;
  has_report_ = rp.do_report != 0;
  if (!locality_used_) {
    steady_src_ = steady_next;
    std::memcpy(steady_ctl_, hctl_, sizeof(steady_ctl_));
  }
  err_bits_ = hctl_[2] & (kErrCandOverflow | kErrSearchOverflow | kErrRounds);
  if (err_bits_ && !isolate_) throw std::runtime_error(error_text(err_bits_));
}

void Matcher::get_trace_errors(uint32_t* out) {
  sync();
  if (n_traces_) RM_HIP(hipMemcpy(out, ws_.trace_err, n_traces_ * 4ull, hipMemcpyDeviceToHost));
}

// report() on host-supplied segment lists, one thread per trace (rm_report_segments)
void report_segments(int device, uint32_t T, const uint32_t* seg_off, const SegmentRec* segs, const double* end_time,
                     const double* threshold, const uint32_t* rmask, const uint32_t* tmask, uint32_t* rep_off,
                     ReportRec* reps, ReportStats* stats) {
  RM_HIP(hipSetDevice(device));
  if (T == 0) { rep_off[0] = 0; return; }
  for (uint32_t k = 0; k < T; ++k)
    if (seg_off[k + 1] < seg_off[k]) throw std::runtime_error("segment offsets not monotone");
  const uint64_t S = seg_off[T];
  std::vector<void*> L;
  struct Free { std::vector<void*>& l; ~Free() { for (void* p : l) (void)hipFree(p); } } fr{L};
  uint32_t* d_off = dalloc<uint32_t>(L, T + 1);
  SegmentRec* d_segs = dalloc<SegmentRec>(L, S);
  double* d_end = dalloc<double>(L, T);
  double* d_thr = dalloc<double>(L, T);
  uint32_t* d_rm = dalloc<uint32_t>(L, T);
  uint32_t* d_tm = dalloc<uint32_t>(L, T);
  ReportRec* d_reps = dalloc<ReportRec>(L, S);
  ReportStats* d_st = dalloc<ReportStats>(L, T);
  RM_HIP(hipMemcpy(d_off, seg_off, (T + 1) * 4ull, hipMemcpyHostToDevice));
  if (S) RM_HIP(hipMemcpy(d_segs, segs, S * sizeof(SegmentRec), hipMemcpyHostToDevice));
  RM_HIP(hipMemcpy(d_end, end_time, T * 8ull, hipMemcpyHostToDevice));
  RM_HIP(hipMemcpy(d_thr, threshold, T * 8ull, hipMemcpyHostToDevice));
  RM_HIP(hipMemcpy(d_rm, rmask, T * 4ull, hipMemcpyHostToDevice));
  RM_HIP(hipMemcpy(d_tm, tmask, T * 4ull, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_report_lists, dim3(T), dim3(64), 0, 0, T, d_off, d_segs, d_end, d_thr, d_rm, d_tm,
                     d_reps, d_st);
  RM_HIP(hipGetLastError());
  std::vector<ReportRec> all(S);
  if (S) RM_HIP(hipMemcpy(all.data(), d_reps, S * sizeof(ReportRec), hipMemcpyDeviceToHost));
  RM_HIP(hipMemcpy(stats, d_st, T * sizeof(ReportStats), hipMemcpyDeviceToHost));
  uint64_t at = 0;
  for (uint32_t k = 0; k < T; ++k) {
    rep_off[k] = (uint32_t)at;
    const uint32_t c = (uint32_t)stats[k].n_reports;
    if (c) std::memcpy(reps + at, all.data() + seg_off[k], c * sizeof(ReportRec));
    at += c;
  }
  rep_off[T] = (uint32_t)at;
}

// ---- downloads ----
void Matcher::get_states(uint32_t* n_states, uint32_t* state_orig) {
  sync();
  RM_HIP(hipMemcpy(n_states, ws_.n_states, n_traces_ * 4ull, hipMemcpyDeviceToHost));
  RM_HIP(hipMemcpy(state_orig, ws_.state_orig, n_points_ * 4, hipMemcpyDeviceToHost));
}
void Matcher::get_candidates(uint8_t* cand_n, uint32_t* road, uint32_t* s_cm, float* sq) {
  sync();
  RM_HIP(hipMemcpy(cand_n, ws_.cand_n, n_points_, hipMemcpyDeviceToHost));
  {
    std::vector<uint4> desc(n_points_ * kMaxCand * 2);
    RM_HIP(hipMemcpy(desc.data(), ws_.cand_desc, desc.size() * sizeof(uint4), hipMemcpyDeviceToHost));
    for (uint64_t x = 0; x < n_points_ * kMaxCand; ++x) { road[x] = desc[2 * x].x; s_cm[x] = desc[2 * x].y; }
  }
  RM_HIP(hipMemcpy(sq, ws_.cand_sq, n_points_ * kMaxCand * 4, hipMemcpyDeviceToHost));
}
void Matcher::get_routes(uint32_t* trans_off, double* gc, uint32_t* route) {
  sync();
  RM_HIP(hipMemcpy(trans_off, ws_.trans_off, n_points_ * 4, hipMemcpyDeviceToHost));
  RM_HIP(hipMemcpy(gc, ws_.gc, n_points_ * 8, hipMemcpyDeviceToHost));
  if (n_trans_) RM_HIP(hipMemcpy(route, ws_.route, n_trans_ * 4, hipMemcpyDeviceToHost));
}
int Matcher::get_route_terms(double* out) {
  sync();
  if (!turn_mask_ || !ws_.route_d) return 0;
  if (n_trans_) RM_HIP(hipMemcpy(out, ws_.route_d, n_trans_ * 8, hipMemcpyDeviceToHost));
  return 1;
}
void Matcher::get_viterbi(int8_t* choice, uint8_t* chain_start) {
  sync();
  RM_HIP(hipMemcpy(choice, ws_.choice, n_points_, hipMemcpyDeviceToHost));
  RM_HIP(hipMemcpy(chain_start, ws_.chain_start, n_points_, hipMemcpyDeviceToHost));
}
void Matcher::get_paths(uint32_t* path_off, uint32_t* path_cnt, uint32_t* pool, uint32_t* route_dist) {
  // device layout: short paths inline per slot, long ones in the pool; returned compacted in slot order
  sync();
  const uint64_t P = n_points_;
  std::vector<uint32_t> off(P), inl(P * kInlinePath), used(1, 0);
  RM_HIP(hipMemcpy(off.data(), ws_.path_off, P * 4, hipMemcpyDeviceToHost));
  RM_HIP(hipMemcpy(path_cnt, ws_.path_cnt, P * 4, hipMemcpyDeviceToHost));
  RM_HIP(hipMemcpy(inl.data(), ws_.path_inline, P * kInlinePath * 4, hipMemcpyDeviceToHost));
  RM_HIP(hipMemcpy(route_dist, ws_.route_dist, P * 4, hipMemcpyDeviceToHost));
  RM_HIP(hipMemcpy(used.data(), ws_.ctl, 4, hipMemcpyDeviceToHost));
  std::vector<uint32_t> dpool(used[0]);
  if (used[0]) RM_HIP(hipMemcpy(dpool.data(), ws_.path_pool, used[0] * 4ull, hipMemcpyDeviceToHost));
  std::vector<uint32_t> choice_ok(P, 0);
  {
    std::vector<int8_t> ch(P);
    std::vector<uint8_t> cs(P);
    RM_HIP(hipMemcpy(ch.data(), ws_.choice, P, hipMemcpyDeviceToHost));
    RM_HIP(hipMemcpy(cs.data(), ws_.chain_start, P, hipMemcpyDeviceToHost));
    std::vector<uint32_t> tro(n_traces_ + 1), ns(n_traces_);
    RM_HIP(hipMemcpy(tro.data(), in_.trace_off, (n_traces_ + 1) * 4ull, hipMemcpyDeviceToHost));
    RM_HIP(hipMemcpy(ns.data(), ws_.n_states, n_traces_ * 4ull, hipMemcpyDeviceToHost));
    for (uint32_t k = 0; k < n_traces_; ++k)
      for (uint32_t s = 1; s < ns[k]; ++s) {
        const uint64_t l = tro[k] + s;
        choice_ok[l] = (!cs[l] && ch[l] >= 0) ? 1u : 0u;
      }
  }
  uint64_t at = 0;
  for (uint64_t p = 0; p < P; ++p) {
    if (!choice_ok[p]) { path_off[p] = (uint32_t)at; path_cnt[p] = 0; continue; }
    const uint32_t n = path_cnt[p];
    path_off[p] = (uint32_t)at;
    const uint32_t* src = n <= (uint32_t)kInlinePath ? inl.data() + p * kInlinePath : dpool.data() + off[p];
    std::memcpy(pool + at, src, n * 4ull);
    at += n;
  }
}

void Matcher::ctl_words(uint32_t* out) {
  sync();
  for (int i = 0; i < kCtlWords; ++i) out[i] = 0;
  if (ws_.ctl && n_traces_) RM_HIP(hipMemcpy(out, ws_.ctl, kCtlWords * sizeof(uint32_t), hipMemcpyDeviceToHost));
}

void Matcher::tier_counts(uint32_t* out4) {
  uint32_t c[kCtlWords];
  ctl_words(c);
  out4[0] = c[3]; out4[1] = c[5]; out4[2] = c[4]; out4[3] = c[7];
}

uint64_t Matcher::count_segments() {
  sync();
  std::vector<uint32_t> cnt(n_traces_);
  if (n_traces_) RM_HIP(hipMemcpy(cnt.data(), ws_.seg_cnt, n_traces_ * 4ull, hipMemcpyDeviceToHost));
  uint64_t t = 0;
  for (uint32_t c : cnt) t += c;
  return t;
}
// grow-only pinned host buffer of the downloads: failing to pin it is a batch too large for
// the host, which the coalescer splits (serve_policy.hpp), not a generic error
void Matcher::grow_dl_host(size_t need) {
  if (need <= dl_host_bytes_) return;
  const size_t want = std::max(need, dl_host_bytes_ + dl_host_bytes_ / 2);
  if (dl_host_) RM_HIP(hipHostFree(dl_host_));
  dl_host_ = nullptr;
  dl_host_bytes_ = 0;
  void* p = nullptr;
  size_t got = want;
  hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
  if (e != hipSuccess && want > need) {
    (void)hipGetLastError();
    got = need;
    e = hipHostMalloc(&p, need, hipHostMallocDefault);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    throw BatchTooLarge("pinned download buffer of " + std::to_string(need) + " bytes: " + hipGetErrorString(e));
  }
  dl_host_ = p;
  dl_host_bytes_ = got;
}

// grow-only device buffer of the downloads (offsets, then the compacted records)
void Matcher::grow_dl_dev(size_t dev_need) {
  if (dev_need <= dl_dev_bytes_) return;
  const size_t want = std::max(dev_need, dl_dev_bytes_ + dl_dev_bytes_ / 2);
  if (dl_dev_) RM_HIP(hipFree(dl_dev_));
  dl_dev_ = nullptr;
  dl_dev_bytes_ = 0;
  // test hook: allocations above RM_TEST_DOWNLOAD_ALLOC_LIMIT bytes fail as out of memory
  // (tests/test_gpu_isolation.py drives the failure and the call after it)
  const char* lim = std::getenv("RM_TEST_DOWNLOAD_ALLOC_LIMIT");
  const size_t limit = lim && *lim ? (size_t)std::strtoull(lim, nullptr, 10) : ~(size_t)0;
  void* p = nullptr;
  size_t got = 0;
  for (const size_t sz : {want, dev_need}) {
    if (sz > limit) continue;
    std::vector<void*> buf;
    try {
      dalloc<char>(buf, sz);
    } catch (const OutOfDeviceMemory&) {
      continue;
    }
    p = buf[0];
    got = sz;
    break;
  }
  if (!p) throw BatchTooLarge("segment download buffer of " + std::to_string(dev_need) + " bytes does not fit in HBM");
  dl_dev_ = p;
  dl_dev_bytes_ = got;
}

void Matcher::download_compacted(const uint32_t* d_base, const uint32_t* d_cnt, const void* d_src, uint32_t words,
                                 uint32_t* off, void* dst, const std::function<void*(uint64_t)>& dst_for) {
  const uint32_t T = n_traces_;
  hipStream_t st = stream_;
  RM_HIP(hipSetDevice(eng_->device()));
  seg_prefetched_ = false;   // the device buffer is reused below
  const size_t offb = ((size_t)T + 1) * 4;
  // pinned: [0, offb) the counts then offsets, then the compacted records
  // The buffers grow by half again (or to the need).  The old buffer is released first and the
  // pointer / size pair only records a buffer that exists, so a failed allocation leaves (null, 0)
  // and the next call allocates again; running out of memory here is a batch too large for the
  // device, which the coalescer splits (serve_policy.hpp), not a generic error.
  grow_dl_host(offb);
  uint32_t* hc = (uint32_t*)dl_host_;
  RM_HIP(hipMemcpyAsync(hc, d_cnt, T * 4ull, hipMemcpyDeviceToHost, st));
  RM_HIP(hipStreamSynchronize(st));
  uint64_t at = 0;
  for (uint32_t k = 0; k < T; ++k) {
    off[k] = (uint32_t)at;
    at += hc[k];
  }
  off[T] = (uint32_t)at;
  if (dst_for) dst = dst_for(at);   // the caller sizes its buffer from the total
  if (at == 0) return;
  const size_t recb = (size_t)at * words * 8;
  const size_t dev_need = offb + recb + 8;
  grow_dl_dev(dev_need);
  grow_dl_host(offb + recb + 8);
  hc = (uint32_t*)dl_host_;
  std::memcpy(hc, off, offb);
  uint32_t* d_off = (uint32_t*)dl_dev_;
  unsigned long long* d_dst = (unsigned long long*)((char*)dl_dev_ + ((offb + 7) & ~(size_t)7));
  RM_HIP(hipMemcpyAsync(d_off, hc, offb, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_gather_recs, dim3(std::min<uint32_t>(T, 8192u)), dim3(64), 0, st, T, d_base, d_cnt, d_off,
                     (const unsigned long long*)d_src, words, d_dst);
  char* h_dst = (char*)dl_host_ + ((offb + 7) & ~(size_t)7);
  RM_HIP(hipMemcpyAsync(h_dst, d_dst, recb, hipMemcpyDeviceToHost, st));
  RM_HIP(hipStreamSynchronize(st));
  std::memcpy(dst, h_dst, recb);
}

// a small run's segments, compacted by the run itself (run_small): one copy down
bool Matcher::download_prefetched(uint32_t* off, void* dst, const std::function<void*(uint64_t)>& dst_for) {
  if (!seg_prefetched_) return false;
  seg_prefetched_ = false;   // once: the buffers are shared with the other downloads
  const uint32_t T = n_traces_;
  std::memcpy(off, hoff_, ((size_t)T + 1) * 4);
  const uint64_t at = off[T];
  if (dst_for) dst = dst_for(at);
  if (at == 0) return true;
  const size_t offb = (((size_t)T + 1) * 4 + 7) & ~(size_t)7;
  const size_t recb = (size_t)at * sizeof(SegmentRec);
  grow_dl_host(recb);
  RM_HIP(hipMemcpyAsync(dl_host_, (const char*)dl_dev_ + offb, recb, hipMemcpyDeviceToHost, stream_));
  RM_HIP(hipStreamSynchronize(stream_));
  std::memcpy(dst, dl_host_, recb);
  return true;
}

void Matcher::get_segments(uint32_t* seg_off, SegmentRec* segs) {
  sync();
  if (!n_traces_) { seg_off[0] = 0; return; }
  static_assert(sizeof(SegmentRec) % 8 == 0, "records move as u64 words");
  if (download_prefetched(seg_off, segs, nullptr)) return;
  download_compacted(ws_.seg_base, ws_.seg_cnt, ws_.segs, sizeof(SegmentRec) / 8, seg_off, segs, nullptr);
}
void Matcher::get_segments(std::vector<uint32_t>& seg_off, std::vector<SegmentRec>& segs) {
  sync();
  seg_off.assign((size_t)n_traces_ + 1, 0u);
  segs.clear();
  if (!n_traces_) return;
  if (download_prefetched(seg_off.data(), nullptr, [&](uint64_t n) -> void* {
        segs.resize(n);
        return segs.data();
      }))
    return;
  download_compacted(ws_.seg_base, ws_.seg_cnt, ws_.segs, sizeof(SegmentRec) / 8, seg_off.data(), nullptr,
                     [&](uint64_t n) -> void* {
                       segs.resize(n);
                       return segs.data();
                     });
}
uint64_t Matcher::count_reports() {
  sync();
  if (!has_report_) return 0;
  std::vector<uint32_t> cnt(n_traces_);
  if (n_traces_) RM_HIP(hipMemcpy(cnt.data(), ws_.rep_cnt, n_traces_ * 4ull, hipMemcpyDeviceToHost));
  uint64_t t = 0;
  for (uint32_t c : cnt) t += c;
  return t;
}
void Matcher::get_reports(uint32_t* rep_off, ReportRec* reps, ReportStats* stats) {
  sync();
  if (!has_report_) throw std::runtime_error("the last run did not compute reports");
  if (!n_traces_) { rep_off[0] = 0; return; }
  RM_HIP(hipMemcpy(stats, ws_.stats, n_traces_ * sizeof(ReportStats), hipMemcpyDeviceToHost));
  static_assert(sizeof(ReportRec) % 8 == 0, "records move as u64 words");
  download_compacted(ws_.seg_base, ws_.rep_cnt, ws_.reps, sizeof(ReportRec) / 8, rep_off, reps, nullptr);
}

}  // namespace rm
