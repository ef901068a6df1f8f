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
// alone, at the lone-wave latency); part 2 = [d2, n) WIDE on the CUs left over, joined by the
// deep parts' CUs as those finish.  Makespan = max(deep latencies, WIDE drain time, longest
// WIDE job's latency); within 2 % the plan with less total issue work wins.  Measured on the
// mixed config (configs[3]): WIDE waves sharing SIMDs with deep waves lose to them (older
// waves issue first), which is why the deep parts get CUs of their own.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cmath>
#include <numeric>
#include <vector>

#include "efes_internal.hpp"

namespace {

constexpr double kCpiDeep = 4.1;    // cycles per instruction, DEEP / GROUP wave alone
constexpr double kCpiWide = 5.1;    // cycles per instruction, WIDE wave alone (dependent CRC LDS lookups)
// ... and a lone WIDE wave on CUs of its own while the rest of the chip is busy (configs[3] trace:
// the 32 MiB class as an exclusive WIDE part beside FED4 and shared WIDE parts ended at 1.153 s,
// 29 MB/s per lane; profiles/r02_mixtrace/)
constexpr double kCpiWideExclusive = 7.0;
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

struct Cand {
  double t = -1;
  uint32_t d1 = 0, d2 = 0;
  int g0 = 64, g1 = 64;
};

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
  Cand best;
  double best_work = 0;
  for (size_t a = 0; a < cuts.size(); ++a) {
    const uint32_t d1 = cuts[a];
    for (int g0 : shapes) {
      if (g0 == kWideLanes || (d1 == 0 && g0 != 64)) continue;
      double cus0 = 0;
      const double t0 = d1 ? deep_time(g0, 0, d1, &cus0) : 0.0;
      for (size_t b = a; b < cuts.size(); ++b) {
        const uint32_t d2 = cuts[b];
        for (int g1 : shapes) {
          if (d2 == d1 && g1 != 64) continue;
          double cus1 = 0;
          const double t1 = d2 > d1 ? deep_time(g1, d1, d2 - d1, &cus1) : 0.0;
          const bool wide = d2 < n;
          if ((d1 && d2 > d1 && cus0 + cus1 > cus) || (wide && cus0 + cus1 >= cus)) continue;
          double t = std::max(t0, t1);
          double wk = pre[d1] * work(g0, false) + (pre[d2] - pre[d1]) * work(g1, false);
          if (wide) {
            // WIDE work drains through the free SIMDs: 4*(cus - cus0 - cus1) until the shorter
            // deep part ends, then its CUs join, then the other's.
            const double free0 = 4.0 * (cus - cus0 - cus1);
            const double w = waves(kWideLanes, n - d2);
            const double need = (pre[n] - pre[d2]) * work(kWideLanes, w > 1.5 * free0);
            wk += need;
            double ta = d1 ? t0 : 0.0, tb = d2 > d1 ? t1 : 0.0, ca = cus0, cb = cus1;
            if (ta > tb) { std::swap(ta, tb); std::swap(ca, cb); }
            double done = 0, tw = 0;
            const double seg[3][2] = {{ta, free0}, {tb, free0 + 4.0 * ca}, {1e300, 4.0 * cus}};
            double t_prev = 0;
            for (const auto& sg : seg) {
              const double cap = (sg[0] - t_prev) * sg[1];
              if (done + cap >= need) { tw = t_prev + (need - done) / sg[1]; break; }
              done += cap;
              t_prev = sg[0];
            }
            // the longest WIDE job runs alone on its SIMD only if every WIDE wave has one
            const double stretch = w > free0 ? 2.0 / kWideShare : 1.0;
            t = std::max(t, std::max(tw, blocks(d2) * latency(kWideLanes) * stretch));
          }
          // equal makespans (within 2 %): prefer less issue work (fewer busy SIMDs, higher clock)
          if (best.t < 0 || t < best.t * 0.98 || (t < best.t * 1.02 && wk < best_work)) {
            if (best.t < 0 || t < best.t * 1.02) {
              best = Cand{t, d1, d2, g0, g1};
              best_work = wk;
            }
          }
        }
      }
    }
  }

  efes_plan_part parts[EFES_PLAN_MAX_PARTS] = {};
  uint32_t np = 0;
  if (best.d1) parts[np++] = efes_plan_part{best.d1, mode_of(best.g0), 1u, 0u};
  if (best.d2 > best.d1) parts[np++] = efes_plan_part{best.d2 - best.d1, mode_of(best.g1), 1u, 0u};
  if (n > best.d2) parts[np++] = efes_plan_part{n - best.d2, EFES_MODE_WIDE, 0u, 0u};

  // Developer override for calibration runs:
  //   EFES_PLAN_FORCE="<lanes>:<jobs>[x],<lanes>:<jobs>[x],..."  (lanes 64 = DEEP, 0 = WIDE,
  //   1 = FED4, 2 = FED4E (both always exclusive), x = exclusive); jobs beyond the listed parts run WIDE (a fourth
  //   part is not possible).
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
  plan->est_seconds = best.t / kClock;
  return EFES_OK;
}

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
  // Fork: parts 0..k-2 on side streams (longest jobs first, so their workgroups are placed
  // first), the last part on `stream`; join: `stream` waits for every side stream.
  hipError_t e = plan->nparts > 1 ? hipEventRecord(ctx->ev_fork, s) : hipSuccess;
  const efes_job* first = jobs;
  for (uint32_t i = 0; i + 1 < plan->nparts && e == hipSuccess; ++i) {
    e = hipStreamWaitEvent(ctx->side[i], ctx->ev_fork, 0);
    if (e == hipSuccess) e = launch(plan->part[i], first, ctx->side[i]);
    if (e == hipSuccess) e = hipEventRecord(ctx->ev_join[i], ctx->side[i]);
    first += plan->part[i].jobs;
  }
  if (e == hipSuccess) e = launch(plan->part[plan->nparts - 1], first, s);
  for (uint32_t i = 0; i + 1 < plan->nparts && e == hipSuccess; ++i) e = hipStreamWaitEvent(s, ctx->ev_join[i], 0);
  return e == hipSuccess ? EFES_OK : EFES_ERR_HIP;
}

}  // extern "C"
