// efes_plan.cpp -- placement of a mixed-length batch on one GPU (efes_plan_batch) and its
// concurrent multi-part launch (efes_hash_submit_plan).
//
// SHA-1 is a chain per job (sha1.go:129-203 runs block after block), so a batch's makespan is
// at least its longest job's latency, and the kernel shapes trade latency for issue work.
// Per 64-B block, in SIMD cycles (MI355X, measured: DESIGN.md §4 "grouped DEEP"):
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
// alone, at the lone-wave latency); the rest [d2, n) WIDE on the CUs left over, joined by the
// exclusive parts' CUs as those finish.  The best such plan may then take a third exclusive part
// [d2, d3) (e.g. the 16 MiB class of configs[3] as WIDE with one wave per SIMD, whose lanes
// otherwise share SIMDs and set the tail).  Makespan = max(exclusive latencies, WIDE drain time,
// longest WIDE job's latency); within 2 % the plan with less total issue work wins.  Measured on the
// mixed config (configs[3]): WIDE waves sharing SIMDs with deep waves lose to them (older
// waves issue first), which is why the deep parts get CUs of their own.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cmath>
#include <numeric>
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
// jobs per CU and cycles of one 4-block chain super-step (tools/fed_stats.py, DESIGN.md §4 FED)
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

  // cut candidates: where the length changes, thinned to <= 96 by cumulative blocks
  std::vector<uint32_t> cuts{0};
  for (uint32_t i = 1; i < n; ++i)
    if (blocks(i) != blocks(i - 1)) cuts.push_back(i);
  cuts.push_back(n);
  if (cuts.size() > 96) {
    std::vector<uint32_t> thin{0};
    for (int q = 1; q < 95; ++q) {
      const double target = pre[n] * q / 95.0;
      const uint32_t i = (uint32_t)(std::lower_bound(pre.begin(), pre.end(), target) - pre.begin());
      auto it = std::lower_bound(cuts.begin(), cuts.end(), std::min(i, n));
      if (it != cuts.end() && *it != thin.back()) thin.push_back(*it);
    }
    if (thin.back() != n) thin.push_back(n);
    cuts.swap(thin);
  }

  // Every DEEP/GROUP part is exclusive (its workgroups own their CUs, so its waves run alone at
  // the lone-wave latency); WIDE runs on the CUs left over and on those the deep parts free.
  // Part 1 may also be WIDE on CUs of its own (one wave per SIMD: its lanes at the lone-wave rate).
  const int shapes[] = {64, 32, 16, 8, 4, kFed, kFedE, kWideLanes};
  auto deep_time = [&](int g, uint32_t first, uint32_t jobs, double* cus_out) {
    const double c = std::ceil(waves(g, jobs) / 4.0);
    *cus_out = std::min(c, cus);
    const double lat = g == kWideLanes ? 740.0 * kCpiWideExclusive : latency(g);
    return blocks(first) * lat * std::ceil(c / cus);  // rounds of workgroups beyond one per CU
  };
  // Makespan of a candidate: exclusive parts ps[0..k) (jobs [previous end, end) in shape g, on
  // CUs of their own) concurrent with a WIDE part for the remaining jobs, which drains through
  // the CUs left over and is joined by each exclusive part's CUs as that part ends.
  struct Part {
    uint32_t end;
    int g;
  };
  auto evaluate = [&](const Part* ps, int k, double* work_out) -> double {
    double t = 0, wk = 0, used = 0;
    std::pair<double, double> fin[EFES_PLAN_MAX_PARTS];  // (end time, CUs) of each exclusive part
    int nf = 0;
    uint32_t start = 0;
    for (int i = 0; i < k; ++i) {
      if (ps[i].end <= start) continue;
      double c = 0;
      const double ti = deep_time(ps[i].g, start, ps[i].end - start, &c);
      t = std::max(t, ti);
      wk += (pre[ps[i].end] - pre[start]) * work(ps[i].g, false);
      used += c;
      fin[nf++] = {ti, c};
      start = ps[i].end;
    }
    *work_out = wk;
    if (used > cus || (start < n && used >= cus)) return -1;  // does not fit
    if (start < n) {
      const double free0 = 4.0 * (cus - used);
      const double w = waves(kWideLanes, n - start);
      const double need = (pre[n] - pre[start]) * work(kWideLanes, w > 1.5 * free0);
      *work_out += need;
      std::sort(fin, fin + nf);
      double done = 0, tw = -1, t_prev = 0, rate = free0;
      for (int i = 0; i <= nf && tw < 0; ++i) {
        const double t_end = i < nf ? fin[i].first : 1e300;
        const double cap = (t_end - t_prev) * rate;
        if (done + cap >= need) tw = t_prev + (need - done) / rate;
        done += cap;
        t_prev = t_end;
        if (i < nf) rate += 4.0 * fin[i].second;
      }
      // the longest WIDE job runs alone on its SIMD only if every WIDE wave has one
      const double stretch = w > free0 ? 2.0 / kWideShare : 1.0;
      t = std::max(t, std::max(tw, blocks(start) * 740.0 * kCpiWideBusy * stretch));
    }
    return t;
  };
  // equal makespans (within 2 %): prefer less issue work (fewer busy SIMDs, higher clock)
  Part best[EFES_PLAN_MAX_PARTS - 1] = {};
  int best_k = 0;
  double best_t = -1, best_work = 0;
  auto consider = [&](const Part* ps, int k) {
    double wk = 0;
    const double t = evaluate(ps, k, &wk);
    if (t < 0) return;
    if (best_t < 0 || t < best_t * 0.98 || (t < best_t * 1.02 && wk < best_work)) {
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

  // Developer override for calibration runs:
  //   EFES_PLAN_FORCE="<lanes>:<jobs>[x],<lanes>:<jobs>[x],..."  (lanes 64 = DEEP, 0 = WIDE,
  //   1 = FED4, 2 = FED4E (both always exclusive), x = exclusive); jobs beyond the listed parts run
  //   WIDE (a part beyond EFES_PLAN_MAX_PARTS is not possible).
  if (const char* f = getenv("EFES_PLAN_FORCE"); f && *f) {
    efes_plan_part fp[EFES_PLAN_MAX_PARTS] = {};
    uint32_t fn = 0, used = 0;
    bool ok = true;
    for (const char* c = f; *c && ok;) {
      int g = -1, len = 0;
      unsigned long long d = 0;
      ok = sscanf(c, "%d:%llu%n", &g, &d, &len) == 2 && lanes_of(mode_of(g)) == g && fn < EFES_PLAN_MAX_PARTS;
      if (!ok) break;
      c += len;
      const bool x = *c == 'x';
      c += x;
      c += *c == ',';
      const uint32_t take = (uint32_t)std::min<unsigned long long>(d, n - used);
      if (take) fp[fn++] = efes_plan_part{take, mode_of(g), x ? 1u : 0u, 0u};
      used += take;
    }
    if (ok && used < n) {
      if (fn < EFES_PLAN_MAX_PARTS) fp[fn++] = efes_plan_part{n - used, EFES_MODE_WIDE, 0u, 0u};
      else ok = false;
    }
    if (ok) {
      np = fn;
      std::copy(fp, fp + fn, parts);
    }
  }
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
    if (p.mode == EFES_MODE_WIDE) return efes::launch_wide(first, p.jobs, ctx->d_tabs, st, p.exclusive != 0);
    if (p.mode == EFES_MODE_FED4 || p.mode == EFES_MODE_FED4E)
      return efes::launch_fed(first, p.jobs, ctx->d_tabs, st, p.mode == EFES_MODE_FED4E);
    return efes::launch_group(first, p.jobs, lanes_of(p.mode), ctx->d_tabs, st, p.exclusive != 0);
  };
  std::lock_guard<std::mutex> lk(ctx->plan_mu);
  // Fork: part i on the context's part stream i (longest jobs first, so their workgroups are
  // placed first); join: `stream` waits for every part.  The part streams were created one after
  // the other with the context, so they sit on distinct hardware queues (GPU_MAX_HW_QUEUES is 4):
  // a part launched on the caller's stream instead could share a hardware queue with another
  // part and not start before that one ends (seen in kernel traces: profiles/r02_mixtrace/).
  if (plan->nparts == 1) return hip_err_plan(launch(plan->part[0], jobs, s));
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
