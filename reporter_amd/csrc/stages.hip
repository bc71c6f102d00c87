// stages.hip — the GPU stages on either side of the matcher in the reference's batch
// pipeline (reference py/simple_reporter.py):
//
//   run_points   :137-164  raw per-vehicle points -> time sort -> inactivity windows of
//                          >= 2 points, built on the device straight into the matcher's
//                          batch (no host round trip of the points)
//   tiles        :176-196  valid reports -> hour buckets -> CSV rows per tile file
//                :211-254  string order of (id, next_id), privacy cull of short runs,
//                          header + rows; with RCCL the rows of every rank are
//                          all-gathered and each rank emits the files it owns
//
// Sorting uses hipCUB radix sorts (stable), so equal keys keep their input order as the
// reference's stable Python sorts do.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>

#include "engine.hpp"

namespace rm {

namespace {

template <class T>
T* salloc(std::vector<void*>& list, uint64_t n) {
  void* p = nullptr;
  if (n == 0) n = 1;
  RM_HIP(hipMalloc(&p, n * sizeof(T)));
  list.push_back(p);
  return (T*)p;
}

inline uint32_t grid(uint64_t n, uint32_t b = 256) { return (uint32_t)((n + b - 1) / b); }

// ---------------------------------------------------------------- windows
__global__ void k_pt_keys(uint64_t n, const uint32_t* uuid, const double* time, double tbase,
                          unsigned long long* key, uint32_t* val) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double t = floor(time[k]) - tbase;
  key[k] = ((unsigned long long)uuid[k] << 32) | (unsigned long long)(uint32_t)t;
  val[k] = (uint32_t)k;
}

// a window starts at the first point of a vehicle or after a gap > inactivity (:151-153)
__global__ void k_win_flags(uint64_t n, const unsigned long long* key, const uint32_t* perm, const double* time,
                            double inactivity, uint32_t* flag) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  uint32_t f = 1;
  if (k > 0 && (key[k] >> 32) == (key[k - 1] >> 32)) f = (time[perm[k]] - time[perm[k - 1]] > inactivity) ? 1u : 0u;
  flag[k] = f;
}

__global__ void k_win_starts(uint64_t n, const uint32_t* flag, const uint32_t* wid, uint32_t* wstart, uint32_t* hctl) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  if (flag[k]) wstart[wid[k]] = (uint32_t)k;
  if (k + 1 == n) {
    const uint32_t W = wid[k] + flag[k];
    wstart[W] = (uint32_t)n;
    hctl[0] = W;
  }
}

// windows of fewer than 2 points are not matched (:158-160)
__global__ void k_win_sizes(uint32_t W, const uint32_t* wstart, uint32_t* wcnt, uint32_t* wflag) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= W) return;
  const uint32_t size = wstart[w + 1] - wstart[w];
  wcnt[w] = size >= 2 ? size : 0u;
  wflag[w] = size >= 2 ? 1u : 0u;
}

__global__ void k_win_gather(uint64_t n, const unsigned long long* key, const uint32_t* perm, const uint32_t* wid,
                             const uint32_t* wfl, const uint32_t* wstart, const uint32_t* wflag, const uint32_t* wofs, const uint32_t* widx,
                             const double* time, const float* lon, const float* lat, const float* acc,
                             const uint32_t* uopt, uint32_t n_uopt, double* o_time, float* o_lon, float* o_lat,
                             float* o_acc, uint32_t* trace_off, uint32_t* trace_opt, uint32_t* trace_uuid) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t w = wid[k] + wfl[k] - 1u;   // exclusive scan of the start flags -> window of k
  if (!wflag[w]) return;
  const uint32_t src = perm[k];
  const uint32_t dst = wofs[w] + ((uint32_t)k - wstart[w]);
  o_time[dst] = time[src];
  o_lon[dst] = lon[src];
  o_lat[dst] = lat[src];
  o_acc[dst] = acc[src];
  if ((uint32_t)k == wstart[w]) {
    const uint32_t t = widx[w];
    const uint32_t u = (uint32_t)(key[k] >> 32);
    trace_off[t] = dst;
    trace_opt[t] = n_uopt ? uopt[u] : 0u;
    trace_uuid[t] = u;
  }
}

// ---------------------------------------------------------------- tiles
// decimal digits of x as base-11 symbols (digit + 1, 0 after the last digit), 15 places:
// integer order == order of the decimal strings compared character-wise when each is
// followed by ',' (which sorts before every digit), i.e. the reference's string sort
__device__ __forceinline__ unsigned long long dec_key(unsigned long long x, uint32_t* err) {
  uint32_t d[20];
  int nd = 0;
  do { d[nd++] = (uint32_t)(x % 10ull); x /= 10ull; } while (x && nd < 20);
  if (nd > 15) { atomicOr(err, 1u); nd = 15; }
  unsigned long long key = 0;
  for (int i = 0; i < 15; ++i) key = key * 11ull + (i < nd ? (unsigned long long)d[nd - 1 - i] + 1ull : 0ull);
  return key;
}

__device__ __forceinline__ bool row_valid(const ReportRec& r) {  // :177
  const double dt = r.t1 - r.t0;
  return r.t0 > 0 && r.t1 > 0 && dt > 0.5 && r.length > 0 && r.queue_length >= 0;
}

struct TileArgs {
  uint32_t T;
  const uint32_t* trace_off;
  const double* time;
  const ReportRec* reps;
  const uint32_t* seg_base;
  const uint32_t* rep_cnt;
  uint32_t q;
};

// rows per trace; a report spanning more buckets than its window allows is dropped (:184-187)
__global__ void k_tile_count(TileArgs a, uint32_t* cnt) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.T) return;
  const uint32_t o = a.trace_off[k], npt = a.trace_off[k + 1] - o;
  uint32_t rows = 0;
  if (npt) {
    const long long buckets = ((long long)a.time[o + npt - 1] - (long long)a.time[o]) / (long long)a.q + 1;
    const ReportRec* r = a.reps + a.seg_base[k];
    for (uint32_t i = 0; i < a.rep_cnt[k]; ++i) {
      if (!row_valid(r[i])) continue;
      const long long mn = (long long)floor(r[i].t0) / a.q, mx = (long long)ceil(r[i].t1) / a.q;
      if (mx - mn > buckets) continue;
      rows += (uint32_t)(mx - mn + 1);
    }
  }
  cnt[k] = rows;
}

__global__ void k_tile_emit(TileArgs a, const uint32_t* ofs, TileRow* rows) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.T) return;
  const uint32_t o = a.trace_off[k], npt = a.trace_off[k + 1] - o;
  if (!npt) return;
  const long long buckets = ((long long)a.time[o + npt - 1] - (long long)a.time[o]) / (long long)a.q + 1;
  const ReportRec* r = a.reps + a.seg_base[k];
  uint32_t at = ofs[k];
  for (uint32_t i = 0; i < a.rep_cnt[k]; ++i) {
    if (!row_valid(r[i])) continue;
    const long long start = (long long)floor(r[i].t0), end = (long long)ceil(r[i].t1);
    const long long mn = start / a.q, mx = end / a.q;
    if (mx - mn > buckets) continue;
    // Python 2 round() of a positive duration: halves away from zero (:179)
    const double dt = r[i].t1 - r[i].t0;
    const double fl = floor(dt);
    const int32_t dur = (int32_t)fl + ((dt - fl) >= 0.5 ? 1 : 0);
    for (long long b = mn; b <= mx; ++b) {
      TileRow t;
      t.id = r[i].id; t.next_id = r[i].next_id; t.start = start; t.end = end;
      t.duration = dur; t.length = r[i].length; t.queue = r[i].queue_length;
      t.bucket = (uint32_t)b; t.tile = (uint32_t)(r[i].id & 0x1FFFFFFull);
      t.pad[0] = 1u; t.pad[1] = 0u; t.pad[2] = 0u;   // pad[0]: real row (0 = all-gather padding)
      rows[at++] = t;
    }
  }
}

__device__ __forceinline__ unsigned long long file_key(const TileRow& t) {
  return ((unsigned long long)t.bucket << 25) | t.tile;
}

// keep the gathered rows this rank owns (files hashed over ranks, rm_common.hpp tile_file_owner)
__global__ void k_tile_own(uint64_t n, const TileRow* rows, int rank, int nranks, uint32_t* flag) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const TileRow& t = rows[k];
  flag[k] = (t.pad[0] == 1u && tile_file_owner(t.bucket, t.tile, nranks) == rank) ? 1u : 0u;
}

__global__ void k_tile_compact(uint64_t n, const TileRow* src, const uint32_t* flag, const uint32_t* ofs, TileRow* dst) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  if (flag[k]) dst[ofs[k]] = src[k];
}

// sort key pass: 0 = next_id string, 1 = id string, 2 = file (bucket, tile)
__global__ void k_tile_key(uint64_t n, const TileRow* rows, const uint32_t* perm, int which, unsigned long long* key,
                           uint32_t* err) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const TileRow& t = rows[perm[k]];
  key[k] = which == 0 ? dec_key(t.next_id, err) : (which == 1 ? dec_key(t.id, err) : file_key(t));
}

__global__ void k_iota(uint64_t n, uint32_t* v) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) v[k] = (uint32_t)k;
}

// runs of equal (file, id, next_id) in sorted order
__global__ void k_tile_gflags(uint64_t n, const TileRow* rows, const uint32_t* perm, uint32_t* flag) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  uint32_t f = 1;
  if (k > 0) {
    const TileRow& a = rows[perm[k - 1]];
    const TileRow& b = rows[perm[k]];
    f = (file_key(a) != file_key(b) || a.id != b.id || a.next_id != b.next_id) ? 1u : 0u;
  }
  flag[k] = f;
}

__global__ void k_tile_gpos(uint64_t n, const uint32_t* flag, const uint32_t* gid, uint32_t* gpos, uint32_t* hctl) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  if (flag[k]) gpos[gid[k]] = (uint32_t)k;
  if (k + 1 == n) {
    const uint32_t G = gid[k] + flag[k];
    gpos[G] = (uint32_t)n;
    hctl[1] = G;
  }
}

// The reference's cull loop (:221-239) as a rule over the runs of one file: a run is kept
// iff it has >= privacy rows, except that the loop's end-of-list step closes the open run
// together with the final line, so a final run of one row shares the fate of the run
// before it, judged on their joint size (pinned by tests/golden/tiles_golden.json).
__global__ void k_tile_gkeep(uint32_t G, const TileRow* rows, const uint32_t* perm, const uint32_t* gpos,
                             uint32_t privacy, uint8_t* keep) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  auto fkey = [&](uint32_t x) { return file_key(rows[perm[gpos[x]]]); };
  auto size = [&](uint32_t x) { return gpos[x + 1] - gpos[x]; };
  auto file_last = [&](uint32_t x) { return x + 1 == G || fkey(x + 1) != fkey(x); };
  auto file_first = [&](uint32_t x) { return x == 0 || fkey(x - 1) != fkey(x); };
  const uint32_t sz = size(g);
  bool k = sz >= privacy;
  if (file_last(g) && sz == 1 && !file_first(g)) k = size(g - 1) + 1 >= privacy;
  if (!file_last(g) && file_last(g + 1) && size(g + 1) == 1) k = sz + 1 >= privacy;
  keep[g] = k ? 1 : 0;
}

__global__ void k_tile_kflags(uint64_t n, const uint32_t* gid, const uint32_t* gfl, const uint8_t* keep, uint32_t* flag) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) flag[k] = keep[gid[k] + gfl[k] - 1u];   // exclusive scan of run starts -> run of k
}

__global__ void k_tile_out(uint64_t n, const TileRow* rows, const uint32_t* perm, const uint32_t* flag,
                           const uint32_t* ofs, TileRow* out, uint32_t* hctl) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  if (flag[k]) out[ofs[k]] = rows[perm[k]];
  if (k + 1 == n) hctl[2] = ofs[k] + flag[k];
}

void format_row(std::string& o, const TileRow& t, const TileParams& tp) {
  char buf[160];
  std::snprintf(buf, sizeof buf, "%llu,%llu,%d,1,%d,%d,%lld,%lld,", (unsigned long long)t.id,
                (unsigned long long)t.next_id, t.duration, t.length, t.queue, (long long)t.start, (long long)t.end);
  o = buf;
  o += tp.source;
  o += ',';
  o += tp.mode;
  o += '\n';
}

}  // namespace

StageBufs::~StageBufs() {
  for (void* p : allocs) (void)hipFree(p);
  if (hctl) (void)hipHostFree(hctl);
}

static size_t sort_tmp_bytes(uint64_t n, hipStream_t st) {
  size_t a = 0, b = 0;
  RM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, a, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                            (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 64, st));
  RM_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, st));
  return std::max(a, b);
}

void Matcher::ensure_points(uint64_t n, uint32_t n_uuids, uint32_t n_opts) {
  StageBufs& s = sb_;
  if (!s.hctl) RM_HIP(hipHostMalloc((void**)&s.hctl, 16 * sizeof(uint32_t), hipHostMallocDefault));
  if (n <= s.cap_pts && n_uuids <= s.cap_uuids && s.p_opts && n_opts <= 64) return;
  if (n_opts > 64) throw std::runtime_error("at most 64 option sets per point batch");
  // points and rows share nothing; drop the point buffers only
  const uint64_t c = std::max<uint64_t>(n, s.cap_pts) + 64;
  const uint32_t cu = std::max<uint32_t>(n_uuids, s.cap_uuids) + 16;
  auto drop = [&](void*& p) { if (p) { (void)hipFree(p); s.allocs.erase(std::find(s.allocs.begin(), s.allocs.end(), p)); p = nullptr; } };
  void** ptrs[] = {(void**)&s.p_uuid, (void**)&s.p_time, (void**)&s.p_lon, (void**)&s.p_lat, (void**)&s.p_acc,
                   (void**)&s.p_uopt, (void**)&s.p_opts, (void**)&s.k0, (void**)&s.k1, (void**)&s.v0, (void**)&s.v1,
                   (void**)&s.flag, (void**)&s.idx, (void**)&s.wstart, (void**)&s.wcnt, (void**)&s.wofs,
                   (void**)&s.wflag, (void**)&s.widx, (void**)&s.trace_uuid, (void**)&s.tmp};
  for (void** p : ptrs) drop(*p);
  std::vector<void*>& L = s.allocs;
  s.p_uuid = salloc<uint32_t>(L, c); s.p_time = salloc<double>(L, c); s.p_lon = salloc<float>(L, c);
  s.p_lat = salloc<float>(L, c); s.p_acc = salloc<float>(L, c); s.p_uopt = salloc<uint32_t>(L, cu);
  s.p_opts = salloc<MatchOptions>(L, 64);
  s.k0 = salloc<unsigned long long>(L, c); s.k1 = salloc<unsigned long long>(L, c);
  s.v0 = salloc<uint32_t>(L, c); s.v1 = salloc<uint32_t>(L, c);
  s.flag = salloc<uint32_t>(L, c); s.idx = salloc<uint32_t>(L, c); s.wstart = salloc<uint32_t>(L, c + 1);
  s.wcnt = salloc<uint32_t>(L, c); s.wofs = salloc<uint32_t>(L, c); s.wflag = salloc<uint32_t>(L, c);
  s.widx = salloc<uint32_t>(L, c); s.trace_uuid = salloc<uint32_t>(L, c);
  s.tmp_bytes = std::max(s.tmp_bytes, sort_tmp_bytes(std::max<uint64_t>(std::max<uint64_t>(c, s.cap_rows), s.cap_tr), stream_));
  s.tmp = salloc<char>(L, s.tmp_bytes);
  s.cap_pts = c;
  s.cap_uuids = cu;
}

void Matcher::ensure_rows(uint64_t n, uint32_t traces) {
  StageBufs& s = sb_;
  if (!s.hctl) RM_HIP(hipHostMalloc((void**)&s.hctl, 16 * sizeof(uint32_t), hipHostMallocDefault));
  if (!s.derr) s.derr = salloc<uint32_t>(s.allocs, 1);
  if (traces > s.cap_tr || !s.tcnt) {
    auto dropt = [&](uint32_t*& p) { if (p) { (void)hipFree(p); s.allocs.erase(std::find(s.allocs.begin(), s.allocs.end(), (void*)p)); p = nullptr; } };
    dropt(s.tcnt); dropt(s.tofs);
    s.cap_tr = std::max<uint32_t>(traces, s.cap_tr) + 64;
    s.tcnt = salloc<uint32_t>(s.allocs, s.cap_tr);
    s.tofs = salloc<uint32_t>(s.allocs, s.cap_tr);
    if (s.rows) {  // the scan scratch must cover the trace count too
      const size_t need = sort_tmp_bytes(s.cap_tr, stream_);
      if (need > s.tmp_bytes) {
        (void)hipFree(s.tmp); s.allocs.erase(std::find(s.allocs.begin(), s.allocs.end(), s.tmp));
        s.tmp_bytes = need; s.tmp = salloc<char>(s.allocs, need);
      }
    }
  }
  if (n <= s.cap_rows && s.rows) return;
  const uint64_t c = std::max<uint64_t>(n, s.cap_rows) + n / 4 + 1024;
  auto drop = [&](void*& p) { if (p) { (void)hipFree(p); s.allocs.erase(std::find(s.allocs.begin(), s.allocs.end(), p)); p = nullptr; } };
  void** ptrs[] = {(void**)&s.rows, (void**)&s.rows2, (void**)&s.rk, (void**)&s.rk2, (void**)&s.rperm,
                   (void**)&s.rperm2, (void**)&s.rflag, (void**)&s.ridx, (void**)&s.gpos, (void**)&s.gkeep, (void**)&s.tmp};
  for (void** p : ptrs) drop(*p);
  std::vector<void*>& L = s.allocs;
  s.rows = salloc<TileRow>(L, c); s.rows2 = salloc<TileRow>(L, c);
  s.rk = salloc<unsigned long long>(L, c); s.rk2 = salloc<unsigned long long>(L, c);
  s.rperm = salloc<uint32_t>(L, c); s.rperm2 = salloc<uint32_t>(L, c);
  s.rflag = salloc<uint32_t>(L, c); s.ridx = salloc<uint32_t>(L, c);
  s.gpos = salloc<uint32_t>(L, c + 1); s.gkeep = salloc<uint8_t>(L, c);
  s.tmp_bytes = std::max(s.tmp_bytes, sort_tmp_bytes(std::max<uint64_t>(std::max<uint64_t>(c, s.cap_pts), s.cap_tr), stream_));
  s.tmp = salloc<char>(L, s.tmp_bytes);
  s.cap_rows = c;
}

void Matcher::run_points(const PointsDesc& pd, const RunParams& rp) {
  RM_HIP(hipSetDevice(eng_->device()));
  const uint64_t n = pd.n_points;
  from_points_ = true;
  if (n == 0) { n_traces_ = 0; n_points_ = 0; n_trans_ = 0; n_path_ = 0; seg_used_ = 0; return; }
  if (n >= 0xffffffffull) throw std::runtime_error("point batch too large (>= 2^32 points)");
  if (pd.n_opts == 0 || !pd.opts) throw std::runtime_error("point batch needs at least one option set");
  scan_options(pd.opts, pd.n_opts);   // the checks and batch masks of check_batch (turn costs too)
  double tmin = pd.time[0], tmax = pd.time[0];
  for (uint64_t k = 0; k < n; ++k) {
    if (pd.uuid[k] >= pd.n_uuids) throw std::runtime_error("point vehicle index out of range");
    if (!(pd.time[k] == pd.time[k])) throw std::runtime_error("point time is NaN");
    tmin = std::min(tmin, pd.time[k]);
    tmax = std::max(tmax, pd.time[k]);
  }
  if (pd.uuid_opt)
    for (uint32_t u = 0; u < pd.n_uuids; ++u)
      if (pd.uuid_opt[u] >= pd.n_opts) throw std::runtime_error("vehicle option index out of range");
  const double tbase = std::floor(tmin);
  if (std::floor(tmax) - tbase >= 4294967295.0) throw std::runtime_error("point times span more than 2^32 s");
  ensure_points(n, pd.n_uuids, pd.n_opts);
  StageBufs& s = sb_;
  hipStream_t st = stream_;
  RM_HIP(hipMemcpyAsync(s.p_uuid, pd.uuid, n * 4, hipMemcpyHostToDevice, st));
  RM_HIP(hipMemcpyAsync(s.p_time, pd.time, n * 8, hipMemcpyHostToDevice, st));
  RM_HIP(hipMemcpyAsync(s.p_lon, pd.lon, n * 4, hipMemcpyHostToDevice, st));
  RM_HIP(hipMemcpyAsync(s.p_lat, pd.lat, n * 4, hipMemcpyHostToDevice, st));
  if (pd.accuracy) RM_HIP(hipMemcpyAsync(s.p_acc, pd.accuracy, n * 4, hipMemcpyHostToDevice, st));
  else {
    std::vector<float> neg(n, -1.0f);
    RM_HIP(hipMemcpy(s.p_acc, neg.data(), n * 4, hipMemcpyHostToDevice));
  }
  if (pd.uuid_opt) RM_HIP(hipMemcpyAsync(s.p_uopt, pd.uuid_opt, pd.n_uuids * 4ull, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_pt_keys, dim3(grid(n)), dim3(256), 0, st, n, s.p_uuid, s.p_time, tbase, s.k0, s.v0);
  size_t tmp = s.tmp_bytes;
  RM_HIP(hipcub::DeviceRadixSort::SortPairs(s.tmp, tmp, s.k0, s.k1, s.v0, s.v1, (int)n, 0, 64, st));
  hipLaunchKernelGGL(k_win_flags, dim3(grid(n)), dim3(256), 0, st, n, s.k1, s.v1, s.p_time, pd.inactivity, s.flag);
  tmp = s.tmp_bytes;
  RM_HIP(hipcub::DeviceScan::ExclusiveSum(s.tmp, tmp, s.flag, s.idx, (int)n, st));
  hipLaunchKernelGGL(k_win_starts, dim3(grid(n)), dim3(256), 0, st, n, s.flag, s.idx, s.wstart, s.hctl);
  RM_HIP(hipStreamSynchronize(st));
  const uint32_t W = s.hctl[0];
  hipLaunchKernelGGL(k_win_sizes, dim3(grid(W)), dim3(256), 0, st, W, s.wstart, s.wcnt, s.wflag);
  tmp = s.tmp_bytes;
  RM_HIP(hipcub::DeviceScan::ExclusiveSum(s.tmp, tmp, s.wcnt, s.wofs, (int)W, st));
  tmp = s.tmp_bytes;
  RM_HIP(hipcub::DeviceScan::ExclusiveSum(s.tmp, tmp, s.wflag, s.widx, (int)W, st));
  RM_HIP(hipMemcpyAsync(s.hctl + 4, s.wofs + (W - 1), 4, hipMemcpyDeviceToHost, st));
  RM_HIP(hipMemcpyAsync(s.hctl + 5, s.wcnt + (W - 1), 4, hipMemcpyDeviceToHost, st));
  RM_HIP(hipMemcpyAsync(s.hctl + 6, s.widx + (W - 1), 4, hipMemcpyDeviceToHost, st));
  RM_HIP(hipMemcpyAsync(s.hctl + 7, s.wflag + (W - 1), 4, hipMemcpyDeviceToHost, st));
  RM_HIP(hipStreamSynchronize(st));
  const uint64_t P = (uint64_t)s.hctl[4] + s.hctl[5];
  const uint32_t T = s.hctl[6] + s.hctl[7];
  n_traces_ = T;
  n_points_ = P;
  if (T == 0) { n_trans_ = 0; n_path_ = 0; seg_used_ = 0; has_report_ = false; return; }
  ensure(P, T, pd.n_opts);
  use_ws_inputs();
  Workspace& w = ws_;
  RM_HIP(hipMemcpyAsync(w.opts, pd.opts, pd.n_opts * sizeof(MatchOptions), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_win_gather, dim3(grid(n)), dim3(256), 0, st, n, s.k1, s.v1, s.idx, s.flag, s.wstart, s.wflag, s.wofs,
                     s.widx, s.p_time, s.p_lon, s.p_lat, s.p_acc, s.p_uopt, pd.uuid_opt ? pd.n_uuids : 0u, w.time,
                     w.lon, w.lat, w.acc, w.trace_off, w.trace_opt, s.trace_uuid);
  const uint32_t Pu = (uint32_t)P;
  RM_HIP(hipMemcpyAsync(w.trace_off + T, &Pu, 4, hipMemcpyHostToDevice, st));
  RM_HIP(hipStreamSynchronize(st));
  run_device(rp);
}

void Matcher::get_trace_uuid(uint32_t* out) {
  sync();
  if (!from_points_) throw std::runtime_error("the last run did not come from run_points");
  if (n_traces_) RM_HIP(hipMemcpy(out, sb_.trace_uuid, n_traces_ * 4ull, hipMemcpyDeviceToHost));
}

void Matcher::get_batch(uint32_t* trace_off, float* lon, float* lat, double* time, float* acc) {
  sync();
  const uint64_t P = n_points_;
  RM_HIP(hipMemcpy(trace_off, in_.trace_off, (n_traces_ + 1) * 4ull, hipMemcpyDeviceToHost));
  if (!P) return;
  RM_HIP(hipMemcpy(lon, in_.lon, P * 4, hipMemcpyDeviceToHost));
  RM_HIP(hipMemcpy(lat, in_.lat, P * 4, hipMemcpyDeviceToHost));
  RM_HIP(hipMemcpy(time, in_.time, P * 8, hipMemcpyDeviceToHost));
  RM_HIP(hipMemcpy(acc, in_.acc, P * 4, hipMemcpyDeviceToHost));
}

std::string Matcher::tiles(const TileParams& tp, TileComm* comm) {
  sync();
  if (!has_report_) throw std::runtime_error("tiles need a run with the report() epilogue");
  if (tp.quantisation == 0) throw std::runtime_error("quantisation must be positive");
  if (tp.privacy == 0) throw std::runtime_error("privacy must be at least 1");
  RM_HIP(hipSetDevice(eng_->device()));
  StageBufs& s = sb_;
  Workspace& w = ws_;
  hipStream_t st = stream_;
  const uint32_t T = n_traces_;
  ensure_rows(1, T);
  TileArgs a{T, in_.trace_off, in_.time, w.reps, w.seg_base, w.rep_cnt, tp.quantisation};
  // ---- rows of this rank
  uint64_t R = 0;
  if (T) {
    uint32_t* cnt = s.tcnt;
    uint32_t* ofs = s.tofs;
    hipLaunchKernelGGL(k_tile_count, dim3(grid(T, 64)), dim3(64), 0, st, a, cnt);
    size_t tmp = s.tmp_bytes;
    RM_HIP(hipcub::DeviceScan::ExclusiveSum(s.tmp, tmp, cnt, ofs, (int)T, st));
    RM_HIP(hipMemcpyAsync(s.hctl + 8, ofs + (T - 1), 4, hipMemcpyDeviceToHost, st));
    RM_HIP(hipMemcpyAsync(s.hctl + 9, cnt + (T - 1), 4, hipMemcpyDeviceToHost, st));
    RM_HIP(hipStreamSynchronize(st));
    R = (uint64_t)s.hctl[8] + s.hctl[9];
    ensure_rows(R, T);
    if (R) hipLaunchKernelGGL(k_tile_emit, dim3(grid(T, 64)), dim3(64), 0, st, a, ofs, s.rows);
  }
  // ---- RCCL: all-gather every rank's rows, keep the files this rank owns (a one-rank
  // communicator runs the same collectives, so the path is exercised on a single GPU)
  if (comm) {
    const uint64_t Rm = comm->max_u64(R, st);
    const uint64_t all = Rm * (uint64_t)comm->nranks;
    ensure_rows(std::max<uint64_t>(all, 1), T);
    if (all) {
      if (Rm > R) RM_HIP(hipMemsetAsync(s.rows + R, 0, (Rm - R) * sizeof(TileRow), st));   // padding rows: pad[0] = 0
      comm->allgather(s.rows, s.rows2, Rm * sizeof(TileRow), st);
      hipLaunchKernelGGL(k_tile_own, dim3(grid(all)), dim3(256), 0, st, all, s.rows2, comm->rank, comm->nranks, s.rflag);
      size_t tmp = s.tmp_bytes;
      RM_HIP(hipcub::DeviceScan::ExclusiveSum(s.tmp, tmp, s.rflag, s.ridx, (int)all, st));
      hipLaunchKernelGGL(k_tile_compact, dim3(grid(all)), dim3(256), 0, st, all, s.rows2, s.rflag, s.ridx, s.rows);
      RM_HIP(hipMemcpyAsync(s.hctl + 8, s.ridx + (all - 1), 4, hipMemcpyDeviceToHost, st));
      RM_HIP(hipMemcpyAsync(s.hctl + 9, s.rflag + (all - 1), 4, hipMemcpyDeviceToHost, st));
      RM_HIP(hipStreamSynchronize(st));
      R = (uint64_t)s.hctl[8] + s.hctl[9];
    } else {
      R = 0;
    }
  }
  std::string blob;
  if (R == 0) return blob;
  // ---- sort by (file, id string, next_id string): three stable LSD passes
  uint32_t* derr = s.derr;
  RM_HIP(hipMemsetAsync(derr, 0, 4, st));
  hipLaunchKernelGGL(k_iota, dim3(grid(R)), dim3(256), 0, st, R, s.rperm);
  uint32_t* pin = s.rperm;
  uint32_t* pout = s.rperm2;
  for (int pass = 0; pass < 3; ++pass) {
    hipLaunchKernelGGL(k_tile_key, dim3(grid(R)), dim3(256), 0, st, R, s.rows, pin, pass, s.rk, derr);
    size_t tmp = s.tmp_bytes;
    RM_HIP(hipcub::DeviceRadixSort::SortPairs(s.tmp, tmp, s.rk, s.rk2, pin, pout, (int)R, 0, pass == 2 ? 64 : 52, st));
    std::swap(pin, pout);
  }
  const uint32_t* perm = pin;
  // ---- runs, cull rule, compaction in sorted order
  hipLaunchKernelGGL(k_tile_gflags, dim3(grid(R)), dim3(256), 0, st, R, s.rows, perm, s.rflag);
  size_t tmp = s.tmp_bytes;
  RM_HIP(hipcub::DeviceScan::ExclusiveSum(s.tmp, tmp, s.rflag, s.ridx, (int)R, st));
  hipLaunchKernelGGL(k_tile_gpos, dim3(grid(R)), dim3(256), 0, st, R, s.rflag, s.ridx, s.gpos, s.hctl);
  RM_HIP(hipMemcpyAsync(s.hctl + 12, derr, 4, hipMemcpyDeviceToHost, st));
  RM_HIP(hipStreamSynchronize(st));
  if (s.hctl[12]) throw std::runtime_error("segment id with more than 15 decimal digits in a tile row");
  const uint32_t G = s.hctl[1];
  hipLaunchKernelGGL(k_tile_gkeep, dim3(grid(G)), dim3(256), 0, st, G, s.rows, perm, s.gpos, tp.privacy, s.gkeep);
  uint32_t* kflag = pout;  // the spare permutation buffer
  hipLaunchKernelGGL(k_tile_kflags, dim3(grid(R)), dim3(256), 0, st, R, s.ridx, s.rflag, s.gkeep, kflag);
  tmp = s.tmp_bytes;
  RM_HIP(hipcub::DeviceScan::ExclusiveSum(s.tmp, tmp, kflag, s.rflag, (int)R, st));
  hipLaunchKernelGGL(k_tile_out, dim3(grid(R)), dim3(256), 0, st, R, s.rows, perm, kflag, s.rflag, s.rows2, s.hctl);
  RM_HIP(hipStreamSynchronize(st));
  const uint32_t K = s.hctl[2];
  std::vector<TileRow> out(K);
  if (K) RM_HIP(hipMemcpy(out.data(), s.rows2, K * sizeof(TileRow), hipMemcpyDeviceToHost));
  // ---- CSV text per file: header + rows in string order (:241-253)
  static const char* kHeader =
      "segment_id,next_segment_id,duration,count,length,queue_length,minimum_timestamp,maximum_timestamp,source,"
      "vehicle_type\n";
  std::vector<std::string> lines;
  std::string line;
  for (uint32_t i = 0; i < K;) {
    uint32_t j = i;
    lines.clear();
    while (j < K && out[j].bucket == out[i].bucket && out[j].tile == out[i].tile) {
      format_row(line, out[j], tp);
      lines.push_back(line);
      ++j;
    }
    std::sort(lines.begin(), lines.end());
    const uint64_t b = out[i].bucket;
    char name[96];
    std::snprintf(name, sizeof name, "%llu_%llu/%u/%u", (unsigned long long)(b * tp.quantisation),
                  (unsigned long long)((b + 1) * tp.quantisation - 1), out[i].tile & 7u, (out[i].tile >> 3) & 0x3FFFFFu);
    blob += name;
    blob += '\0';
    blob += kHeader;
    for (const std::string& l : lines) blob += l;
    blob += '\0';
    i = j;
  }
  return blob;
}

}  // namespace rm
