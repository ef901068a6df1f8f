// Device enumeration for the native harnesses (not part of the product library): the contexts a
// harness hashes on, opened the way go/hash_gpu.go pool() opens them -- every ordinal below
// efes_device_count(), or the ordinals of an explicit list ("0,0": two contexts of GPU 0, the
// one-GPU rehearsal of a multi-GPU server process) -- skipping and reporting the ones whose
// efes_ctx_create fails, so one bad GPU never hides the others.  A storage server is one process
// using every GPU of its node (server.go:130), so its measurement must be too.
#pragma once

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "efes_hash.h"

struct EfesDevices {
  std::vector<efes_ctx*> ctxs;  // the contexts that opened, in list order
  std::vector<int> ords;        // their HIP ordinals
  int visible = 0;              // efes_device_count()
  int skipped = 0;              // listed ordinals whose context did not open
};

// list: nullptr, "" or "all" = every visible device; else comma-separated ordinals.
inline EfesDevices efes_open_devices(const char* list) {
  EfesDevices d;
  d.visible = efes_device_count();
  std::vector<int> want;
  if (!list || !*list || !strcmp(list, "all")) {
    for (int i = 0; i < d.visible; ++i) want.push_back(i);
  } else {
    for (const char* p = list; *p;) {
      char* end;
      const long v = strtol(p, &end, 10);
      if (end == p) break;
      want.push_back((int)v);
      p = *end == ',' ? end + 1 : end;
    }
  }
  for (int ord : want) {
    efes_ctx* c = nullptr;
    const int rc = efes_ctx_create(ord, &c);
    if (rc != EFES_OK) {
      fprintf(stderr, "device %d skipped: %s\n", ord, efes_strerror(rc));
      ++d.skipped;
      continue;
    }
    d.ctxs.push_back(c);
    d.ords.push_back(ord);
  }
  return d;
}

inline void efes_close_devices(EfesDevices& d) {
  for (efes_ctx* c : d.ctxs) efes_ctx_destroy(c);
  d.ctxs.clear();
}

// Per-device counters as a JSON array: [{"ordinal": o, "launches": .., "jobs": .., "bytes": ..}, ...]
// from before/after snapshots of each context's queue stats.
inline std::string efes_devices_json(const EfesDevices& d, const std::vector<efes_queue_stats>& a,
                                     const std::vector<efes_queue_stats>& b) {
  std::string s = "[";
  for (size_t i = 0; i < d.ords.size(); ++i) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s{\"ordinal\": %d, \"launches\": %llu, \"jobs\": %llu, \"bytes\": %llu}", i ? ", " : "",
             d.ords[i], (unsigned long long)(b[i].launches - a[i].launches),
             (unsigned long long)(b[i].jobs - a[i].jobs), (unsigned long long)(b[i].bytes - a[i].bytes));
    s += buf;
  }
  return s + "]";
}
