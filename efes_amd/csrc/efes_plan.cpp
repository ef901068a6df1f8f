// efes_plan.cpp -- placement of a mixed-length batch on one GPU (efes_plan_batch) and its
// concurrent multi-part launch (efes_hash_submit_plan).
//
// SHA-1 is a chain per job (sha1.go:129-203 runs block after block), so a batch's makespan is
// at least its longest job's latency, and the kernel shapes trade latency for issue work.
// Per 64-B block, in SIMD cycles (MI355X, measured: DESIGN_NOTES.md §4 "grouped DEEP"):
//   shape                      latency of one job           SIMD work per job
//   DEEP  (one wave per job)   422 x 4.1                    422 x 4.1
//   GROUPn (64/n jobs / wave)  (410 + o_n/n) x 4.1          (410 n + o_n)/64 x 4.1
//   (o_n = 665: instructions per super-step besides the chain, measured for n = 4..32)
//   WIDE  (one lane per job)   740 x 5.1                    740/64 x 5.1 (/1.06 once SIMDs hold 2+ waves)
//   FED4  (32 jobs per CU)     427 x 4.1                    4 SIMDs x 7005 cyc / (32 jobs x 4 blocks)
//         (grouped G = 4 with loads/CRC/expansion on two producer SIMDs: DEEP's latency, 1/32 CU
//          per job; measured 7005 cycles per 4-block super-step, 48.5 ms per 4 MiB job)
// A DEEP/GROUP wave issues at ~4.1 cycles per instruction alone and gains almost nothing from
// a second wave on its SIMD (1.06x), so where a long job's wave lands matters: the plan can
// give the longest jobs CUs of their own (exclusive launch) and run the rest on the others.
//
// Search: longest-first order; cuts d1 <= d2 at length boundaries; part 0 = jobs [0, d1) in
// shape g0 and part 1 = [d1, d2) in shape g1, each on CUs of its own (exclusive: its waves run
// alone, at the lone-wave latency); the rest [d2, n) WIDE on the CUs left over, joined by each
// CU of the exclusive parts as that CU's last workgroup ends.  An exclusive part gets
// min(its workgroups, the CUs not yet taken) CUs and runs in rounds when it has more workgroups
// than that: its workgroups are dealt longest-first to the earliest free CU (an LPT schedule,
// as the dispatcher places them), so a part may hold several length classes -- on configs[3]
// FED4E takes the 64 MiB class and GROUP4 the 32, 16 and 8 MiB classes in rounds on the other
// 130 CUs, leaving the rest to WIDE once they free (0.887 s measured, against 0.99 s for GROUP4
// on the 32 MiB class alone with a WIDE part that ends last).  The best such plan may then take
// a third exclusive part [d2, d3).  Makespan = max(exclusive parts' ends, WIDE drain time,
// the longest WIDE job's latency from when the WIDE part gets its first CU); within 0.5 % the
// plan with less total issue work wins.  Measured on the mixed config (configs[3]): WIDE waves
// sharing SIMDs with deep waves lose to them (older waves issue first), which is why the deep
// parts get CUs of their own.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cmath>
#include <numeric>
#include <tuple>
#include <unordered_map>
#include <utility>
#include <vector>

#include "efes_internal.hpp"

namespace {

constexpr double kCpiDeep = 4.1;    // cycles per instruction, DEEP / GROUP wave alone
constexpr double kCpiWide = 5.1;    // cycles per instruction, WIDE wave alone (dependent CRC LDS lookups)
// ... and a lone WIDE wave on CUs of its own while the rest of the chip is busy (configs[3] trace:
// the 32 MiB class as an exclusive WIDE part beside FED4 and shared WIDE parts ended at 1.153 s,
// 29 MB/s per lane; profiles/r02_mixtrace/)
constexpr double kCpiWideExclusive = 7.0;
// ... and the longest lane of the shared WIDE part on the busy chip, before the x2/1.06 stretch
// of sharing its SIMD (configs[3] trace: the 16 MiB class of the shared part ended at 0.976 s;
// profiles/r02_mixtrace/2_6019x-4_6027x.csv)
constexpr double kCpiWideBusy = 6.0;
constexpr double kWideShare = 1.06; // WIDE throughput of a SIMD holding two waves vs one
constexpr double kClock = 2.36e9;   // Hz (GRBM_GUI_ACTIVE during DEEP), for est_seconds only
constexpr int kWideLanes = 0;       // "shape" id of WIDE in the search
constexpr int kFed = 1;             // "shape" id of FED4 (EFES_MODE_FED4)
constexpr int kFedE = 2;            // "shape" id of FED4E (EFES_MODE_FED4E)
// jobs per CU and cycles of one 4-block chain super-step (tools/fed_stats.py, DESIGN_NOTES.md §4 FED)
constexpr double fed_jobs_per_cu(int g) { return g == kFed ? 32.0 : 48.0; }
constexpr double fed_cycles_per_step(int g) { return g == kFed ? 7005.0 : 8219.0; }
constexpr bool is_fed(int g) { return g == kFed || g == kFedE; }

double step_overhead(int) { return 665.0; }
double latency(int g) {  // cycles per block of one job
  if (g == kWideLanes) return 740.0 * kCpiWide;
  if (is_fed(g)) return fed_cycles_per_step(g) / 4.0;
  return (g == 64 ? 408.0 : 410.0 + step_overhead(g) / g) * kCpiDeep;  // DEEP: 46.4 ms per 4 MiB
}
double work(int g, bool crowded) {  // SIMD cycles per block per job
  if (g == kWideLanes) return 740.0 / 64.0 * kCpiWide / (crowded ? kWideShare : 1.0);
  if (is_fed(g)) return 4.0 * fed_cycles_per_step(g) / (fed_jobs_per_cu(g) * 4.0);
  return (g == 64 ? 422.0 : (410.0 * g + step_overhead(g)) / 64.0) * kCpiDeep;
}
// Waves of a deep part (FED4: its chain waves count as half a workgroup's four SIMDs each).
double waves(int g, double jobs) {
  if (is_fed(g)) return 4.0 * std::ceil(jobs / fed_jobs_per_cu(g));
  return std::ceil(jobs / (g == kWideLanes ? 64.0 : 64.0 / g));
}
int mode_of(int g) {
  switch (g) {
    case kWideLanes: return EFES_MODE_WIDE;
    case kFed: return EFES_MODE_FED4;
    case kFedE: return EFES_MODE_FED4E;
    case 4: return EFES_MODE_GROUP4;
    case 8: return EFES_MODE_GROUP8;
    case 16: return EFES_MODE_GROUP16;
    case 32: return EFES_MODE_GROUP32;
    default: return EFES_MODE_DEEP;
  }
}
int lanes_of(int mode) {
  if (mode == EFES_MODE_DEEP) return 64;
  if (mode == EFES_MODE_WIDE) return kWideLanes;
  if (mode == EFES_MODE_FED4) return kFed;
  if (mode == EFES_MODE_FED4E) return kFedE;
  return efes::group_of_mode(mode);
}


}  // namespace

extern "C" {

int efes_plan_batch(efes_ctx* ctx, const uint64_t* lengths, uint32_t n, uint32_t* order, efes_plan* plan) {
  if (!plan || (n && (!lengths || !order)) || n > EFES_MAX_JOBS) return EFES_ERR_ARG;
  *plan = efes_plan{};
  plan->njobs = n;
  if (n == 0) return EFES_OK;
  std::vector<uint32_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0u);
  std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return lengths[a] > lengths[b]; });
  std::copy(idx.begin(), idx.end(), order);

  std::vector<double> pre(n + 1, 0.0);  // prefix sums of 64-B blocks, longest-first
  for (uint32_t i = 0; i < n; ++i) pre[i + 1] = pre[i] + (double)(lengths[idx[i]] >> 6);
  auto blocks = [&](uint32_t i) { return i < n ? (double)(lengths[idx[i]] >> 6) : 0.0; };
  const double cus = ctx ? (double)ctx->cus : 256.0;

  // cut candidates: where the length changes, thinned to <= 64 by cumulative blocks
  std::vector<uint32_t> cuts{0};
  for (uint32_t i = 1; i < n; ++i)
    if (blocks(i) != blocks(i - 1)) cuts.push_back(i);
  cuts.push_back(n);
  if (cuts.size() > 64) {
    std::vector<uint32_t> thin{0};
    for (int q = 1; q < 63; ++q) {
      const double target = pre[n] * q / 63.0;
      const uint32_t i = (uint32_t)(std::lower_bound(pre.begin(), pre.end(), target) - pre.begin());
      auto it = std::lower_bound(cuts.begin(), cuts.end(), std::min(i, n));
      if (it != cuts.end() && *it != thin.back()) thin.push_back(*it);
    }
    if (thin.back() != n) thin.push_back(n);
    cuts.swap(thin);
  }

  // Every DEEP/GROUP part is exclusive (its workgroups own their CUs, so its waves run alone at
  // the lone-wave latency); WIDE runs on the CUs left over and on those the deep parts free.
  // A part may also be WIDE on CUs of its own (one wave per SIMD: its lanes at the lone-wave rate).
  const int shapes[] = {64, 32, 16, 8, 4, kFed, kFedE, kWideLanes};
  // next[i]: the first job after i (longest-first) with fewer blocks than job i.
  std::vector<uint32_t> next(n);
  for (uint32_t i = n; i-- > 0;) next[i] = (i + 1 < n && blocks(i + 1) == blocks(i)) ? next[i + 1] : i + 1;
  auto jobs_per_wg = [](int g) -> uint32_t {  // one workgroup per CU when exclusive
    if (is_fed(g)) return (uint32_t)fed_jobs_per_cu(g);
    if (g == kWideLanes) return 256u;  // four WIDE waves, one per SIMD
    return 4u * (64u / (uint32_t)g);   // DEEP: 4 jobs; GROUPn: four waves of 64/n jobs
  };
  struct Bucket {  // n CUs free from time t on
    double t, n;
  };
  // An exclusive part [first, end) in shape g on c CUs: its workgroups (consecutive jobs,
  // longest first, so a workgroup lasts as long as its first job's chain) are dealt to the
  // earliest free CU, as the dispatcher does; returns the part's end and, in `out`, the times
  // its CUs become free for the WIDE part.  Workgroups are dealt in bulk by runs of equal length
  // (lengths within 12 % of a run's first count as the run's: the model errs long; at most ~55
  // runs between 64 KiB and 64 MiB), so a part costs O(runs x distinct free times) whatever its
  // job count.
  auto lpt = [&](int g, uint32_t first, uint32_t end, double c, std::vector<Bucket>& out) -> double {
    // `out` stays sorted by time; out[head..] are the CUs still to be dealt workgroups.
    out.assign(1, Bucket{0.0, c});
    size_t head = 0;
    const uint32_t per = jobs_per_wg(g);
    const double lat = g == kWideLanes ? 740.0 * kCpiWideExclusive : latency(g);
    double tend = 0;
    for (uint32_t w = first; w < end;) {
      uint32_t run = std::min(next[w], end);  // jobs [w, run) within 12 % of w's length
      while (run < end && blocks(run) >= 0.88 * blocks(w)) run = std::min(next[run], end);
      const uint32_t wgs = (run - w + per - 1) / per;  // workgroups starting in the run
      const double d = blocks(w) * lat;
      double left = wgs;
      while (left > 0) {
        Bucket& e = out[head];  // the earliest free CUs
        const double take = std::min(left, e.n), t1 = e.t + d;
        e.n -= take;
        if (e.n <= 0) ++head;
        auto pos = std::lower_bound(out.begin() + (ptrdiff_t)head, out.end(), t1,
                                    [](const Bucket& x, double t) { return x.t < t; });
        if (pos != out.end() && pos->t == t1) pos->n += take;
        else out.insert(pos, Bucket{t1, take});
        tend = std::max(tend, t1);
        left -= take;
      }
      w += wgs * per;
    }
    out.erase(out.begin(), out.begin() + (ptrdiff_t)head);
    return tend;
  };
  struct Lpt {
    double tend;
    std::vector<Bucket> frees;
  };
  struct KeyHash {
    size_t operator()(const std::tuple<int, uint32_t, uint32_t, int>& k) const {
      return std::hash<uint64_t>()(((uint64_t)std::get<1>(k) * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)std::get<2>(k) << 20) ^
                                   ((uint64_t)std::get<0>(k) << 8) ^ (uint64_t)std::get<3>(k));
    }
  };
  std::unordered_map<std::tuple<int, uint32_t, uint32_t, int>, Lpt, KeyHash> lpt_cache;
  auto lpt_cached = [&](int g, uint32_t first, uint32_t end, double c) -> const Lpt& {
    const auto key = std::make_tuple(g, first, end, (int)c);
    auto it = lpt_cache.find(key);
    if (it != lpt_cache.end()) return it->second;
    Lpt r;
    r.tend = lpt(g, first, end, c, r.frees);
    return lpt_cache.emplace(key, std::move(r)).first->second;
  };
  // Makespan of a candidate: exclusive parts ps[0..k) (jobs [previous end, end) in shape g, each
  // on min(its workgroups, CUs not yet taken) CUs, in rounds when it has more workgroups than
  // that) concurrent with a WIDE part for the remaining jobs, which drains through the CUs left
  // over and is joined by each CU of an exclusive part as that CU's last workgroup ends.
  struct Part {
    uint32_t end;
    int g;
  };
  Part best[EFES_PLAN_MAX_PARTS - 1] = {};
  int best_k = 0;
  double best_t = -1, best_work = 0;
  std::vector<Bucket> frees;
  auto evaluate = [&](const Part* ps, int k, double* work_out) -> double {
    double t = 0, wk = 0, used = 0;
    frees.clear();
    uint32_t start = 0;
    for (int i = 0; i < k; ++i) {
      if (ps[i].end <= start) continue;
      const double need = std::ceil(waves(ps[i].g, ps[i].end - start) / 4.0);
      const double c = std::min(need, cus - used);
      if (c < 1) return -1;  // no CU left for this part
      // a part's lower bound (its longest chain) already above the best plan: not worth an LPT
      // ... nor its work spread over the CUs it gets
      const double lat_i = ps[i].g == kWideLanes ? 740.0 * kCpiWideExclusive : latency(ps[i].g);
      const double lb = std::max(blocks(start) * lat_i,
                                 (pre[ps[i].end] - pre[start]) * lat_i / (double)jobs_per_wg(ps[i].g) / c);
      if (best_t > 0 && lb > best_t * 1.005) return -1;
      const Lpt& r = lpt_cached(ps[i].g, start, ps[i].end, c);
      t = std::max(t, r.tend);
      wk += (pre[ps[i].end] - pre[start]) * work(ps[i].g, false);
      used += c;
      const size_t mid = frees.size();  // both runs sorted by time: merge, not sort
      frees.insert(frees.end(), r.frees.begin(), r.frees.end());
      std::inplace_merge(frees.begin(), frees.begin() + (ptrdiff_t)mid, frees.end(),
                         [](const Bucket& x, const Bucket& y) { return x.t < y.t; });
      start = ps[i].end;
    }
    *work_out = wk;
    if (start < n) {
      const double free0 = 4.0 * (cus - used);  // SIMDs
      if (free0 <= 0 && frees.empty()) return -1;
      const double w = waves(kWideLanes, n - start);
      const double need = (pre[n] - pre[start]) * work(kWideLanes, w > 1.5 * std::max(free0, 4.0));
      *work_out += need;
      double done = 0, tw = -1, t_prev = 0, rate = free0;
      double t_first = free0 > 0 ? 0.0 : -1, simds_first = free0;  // when the WIDE part starts
      for (size_t i = 0; i <= frees.size() && tw < 0; ++i) {
        const double t_end = i < frees.size() ? frees[i].t : 1e300;
        const double cap = (t_end - t_prev) * rate;
        if (rate > 0 && done + cap >= need) tw = t_prev + (need - done) / rate;
        done += cap;
        t_prev = t_end;
        if (i < frees.size()) {
          rate += 4.0 * frees[i].n;
          if (t_first < 0) {
            t_first = frees[i].t;
            simds_first = 4.0 * frees[i].n;
          }
        }
      }
      // the longest WIDE job runs alone on its SIMD only if every WIDE wave has one
      const double stretch = w > simds_first ? 2.0 / kWideShare : 1.0;
      t = std::max(t, std::max(tw, t_first + blocks(start) * 740.0 * kCpiWideBusy * stretch));
    }
    return t;
  };
  // equal makespans (within 0.5 %): prefer less issue work (fewer busy SIMDs, higher clock)
  auto consider = [&](const Part* ps, int k) {
    double wk = 0;
    const double t = evaluate(ps, k, &wk);
    if (t < 0) return;
    if (best_t < 0 || t < best_t * 0.995 || (t < best_t * 1.005 && wk < best_work)) {
      std::copy(ps, ps + k, best);
      best_k = k;
      best_t = t;
      best_work = wk;
    }
  };
  for (size_t a = 0; a < cuts.size(); ++a) {  // two exclusive parts (either may be empty)
    for (int g0 : shapes) {
      if (g0 == kWideLanes || (cuts[a] == 0 && g0 != 64)) continue;
      for (size_t b = a; b < cuts.size(); ++b)
        for (int g1 : shapes) {
          if (cuts[b] == cuts[a] && g1 != 64) continue;
          const Part ps[2] = {{cuts[a], g0}, {cuts[b], g1}};
          consider(ps, 2);
        }
    }
  }
  if (best_k == 2 && best[1].end > best[0].end && best[1].end < n) {  // a third one after the best two
    const Part two[2] = {best[0], best[1]};
    for (uint32_t d3 : cuts) {
      if (d3 <= two[1].end) continue;
      for (int g2 : shapes) {
        const Part ps[3] = {two[0], two[1], {d3, g2}};
        consider(ps, 3);
      }
    }
  }

  efes_plan_part parts[EFES_PLAN_MAX_PARTS] = {};
  uint32_t np = 0, prev = 0;
  for (int i = 0; i < best_k; ++i) {
    if (best[i].end > prev) parts[np++] = efes_plan_part{best[i].end - prev, mode_of(best[i].g), 1u, 0u};
    prev = std::max(prev, best[i].end);
  }
  if (n > prev) parts[np++] = efes_plan_part{n - prev, EFES_MODE_WIDE, 0u, 0u};

  plan->nparts = np;
  std::copy(parts, parts + np, plan->part);
  plan->est_seconds = best_t / kClock;
  return EFES_OK;
}

static int hip_err_plan(hipError_t e) { return e == hipSuccess ? EFES_OK : EFES_ERR_HIP; }

int efes_hash_submit_plan(efes_ctx* ctx, const efes_job* jobs, const efes_plan* plan, void* stream) {
  if (!ctx || !plan || plan->nparts > EFES_PLAN_MAX_PARTS || (plan->njobs && !jobs) || plan->njobs > EFES_MAX_JOBS)
    return EFES_ERR_ARG;
  uint64_t total = 0;
  for (uint32_t i = 0; i < plan->nparts; ++i) {
    const efes_plan_part& p = plan->part[i];
    if (p.mode != EFES_MODE_WIDE && p.mode != EFES_MODE_DEEP && p.mode != EFES_MODE_FED4 &&
        p.mode != EFES_MODE_FED4E && !efes::group_of_mode(p.mode))
      return EFES_ERR_ARG;
    total += p.jobs;
  }
  if (total != plan->njobs) return EFES_ERR_ARG;
  if (plan->njobs == 0) return EFES_OK;
  efes::DeviceGuard guard(ctx->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  auto launch = [&](const efes_plan_part& p, const efes_job* first, hipStream_t st) {
    if (p.mode == EFES_MODE_WIDE) return efes::launch_wide(first, p.jobs, ctx->d_tabs, st, p.exclusive != 0, ctx->cus);
    if (p.mode == EFES_MODE_FED4 || p.mode == EFES_MODE_FED4E)
      return efes::launch_fed(first, p.jobs, ctx->d_tabs, st, p.mode == EFES_MODE_FED4E);
    return efes::launch_group(first, p.jobs, lanes_of(p.mode), ctx->d_tabs, st, p.exclusive != 0);
  };
  std::lock_guard<std::mutex> lk(ctx->plan_mu);
  // Fork: part i on the context's part stream i (longest jobs first, so their workgroups are
  // placed first); join: `stream` waits for every part.  Each part has a stream of its own, never
  // the caller's or the context's NULL stream: a part launched on the caller's stream shared a
  // hardware queue with another part in one trace and did not start before that one ended
  // (profiles/r02_mixtrace/).  HIP assigns hardware queues (GPU_MAX_HW_QUEUES, 4 here)
  // round-robin over every stream of the process, so distinct queues are likely -- the part
  // streams are created one after the other -- but not guaranteed.
  if (plan->nparts == 1) return hip_err_plan(launch(plan->part[0], jobs, s));
  // The part streams, created on the first multi-part plan (plan_mu held).  They must land on
  // distinct hardware queues, or parts meant to run side by side serialize (configs[3] in a fresh
  // process: 1.03-1.09 s per step on ordinary streams, 0.885 s on CU-masked streams, which get a
  // queue each; DESIGN_NOTES.md §4).  A driver that refuses CU masking still gets ordinary streams.
  for (int i = 0; i < EFES_PLAN_MAX_PARTS; ++i)
    if (!ctx->side[i] && efes::own_queue_stream(ctx, &ctx->side[i]) != hipSuccess &&
        hipStreamCreateWithFlags(&ctx->side[i], hipStreamNonBlocking) != hipSuccess) {
      ctx->side[i] = nullptr;
      return EFES_ERR_HIP;
    }
  hipError_t e = hipEventRecord(ctx->ev_fork, s);
  const efes_job* first = jobs;
  for (uint32_t i = 0; i < plan->nparts && e == hipSuccess; ++i) {
    hipStream_t ps = ctx->part_stream(i);
    if (ps != s) e = hipStreamWaitEvent(ps, ctx->ev_fork, 0);
    if (e == hipSuccess) e = launch(plan->part[i], first, ps);
    if (e == hipSuccess && ps != s) e = hipEventRecord(ctx->ev_join[i], ps);
    first += plan->part[i].jobs;
  }
  for (uint32_t i = 0; i < plan->nparts && e == hipSuccess; ++i)
    if (ctx->part_stream(i) != s) e = hipStreamWaitEvent(s, ctx->ev_join[i], 0);
  return e == hipSuccess ? EFES_OK : EFES_ERR_HIP;
}

}  // extern "C"
