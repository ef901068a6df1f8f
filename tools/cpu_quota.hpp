// Benchmark-environment helper for the native drivers (not part of the product library).
//
// The GPU box grants this job 16 CPUs of time (cgroup v2 cpu.max, e.g. "1600000 100000") on a
// machine that shows all of its cores to the process.  Hundreds of runnable request threads
// then run on hundreds of cores at once, use up the period's quota within a few ms, and the
// whole cgroup is throttled for the rest of the 100 ms period (CFS bandwidth control): kernel
// traces showed the GPU idle for ~90 ms out of every ~100.  Pinning the process to as many CPUs
// as the quota grants turns that into ordinary time sharing.  A server deployment does the same
// by sizing its worker threads to its CPU allowance (for the Go reference: GOMAXPROCS).
#pragma once

#include <sched.h>
#include <stdio.h>

#include <algorithm>
#include <cmath>

// Returns the number of CPUs pinned to (0: no quota, nothing changed).
inline int pin_to_cpu_quota() {
  FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r");
  if (!f) return 0;
  char q[32] = {0};
  long period = 0;
  const int got = fscanf(f, "%31s %ld", q, &period);
  fclose(f);
  if (got != 2 || q[0] == 'm' || period <= 0) return 0;  // "max": no quota
  const int want = std::max(1, (int)std::ceil(atof(q) / (double)period));
  cpu_set_t cur, pin;
  if (sched_getaffinity(0, sizeof cur, &cur) != 0 || CPU_COUNT(&cur) <= want) return 0;
  CPU_ZERO(&pin);
  int n = 0;
  for (int c = 0; c < CPU_SETSIZE && n < want; ++c)
    if (CPU_ISSET(c, &cur)) {
      CPU_SET(c, &pin);
      ++n;
    }
  return sched_setaffinity(0, sizeof pin, &pin) == 0 ? n : 0;
}
