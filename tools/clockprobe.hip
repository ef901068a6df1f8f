// clockprobe.hip -- the effective engine clock over a timed region, read on the GPU itself
// (bench.py's `clock` objects; measurement infrastructure, not part of libefeshash).
//
// Two tiny marker launches on the measured stream bracket the region: each of their 1024 one-wave
// workgroups (about four on every CU) records where it ran (XCC_ID and HW_ID: SE, SH, CU), s_memtime
// and s_memrealtime (the 100 MHz constant clock).  s_memtime counters of different units carry
// different offsets (up to ~10 ms between units of one XCD, measured), so start and end marks are
// matched by the CU they ran on: the memtime ticks between them over the realtime between them is
// the clock that CU ran at meanwhile, and the result is the median over the matched CUs.  The marks
// are ordinary kernels in stream order -- nothing runs beside the measured work, nothing waits on
// the host.  Calibration against GRBM_GUI_ACTIVE and amdsmi: profiles/r05_clock/.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <map>
#include <vector>

namespace {

constexpr int kMarkBlocks = 1024;  // dealt over the 256 CUs

__global__ void clock_mark_kernel(unsigned long long* out) {
  if (threadIdx.x != 0) return;
  unsigned xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  const unsigned long long r = __builtin_amdgcn_s_memrealtime();
  unsigned long long* o = out + 3 * blockIdx.x;
  o[0] = (unsigned long long)(xcc & 0xfu) << 16 | ((hw >> 8) & 0xffu);  // XCD, SE, SH, CU
  o[1] = t;
  o[2] = r;
}

unsigned long long* g_marks[64] = {};  // per device: [2][kMarkBlocks][3]

}  // namespace

extern "C" {

// Records mark `which` (0 = start, 1 = end) on `stream` of `device` (the current device is kept).
int clockprobe_mark(int device, void* stream, int which) {
  if (device < 0 || device >= 64 || (which != 0 && which != 1)) return -1;
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) return -2;
  int rc = 0;
  if (!g_marks[device] &&
      hipMalloc(reinterpret_cast<void**>(&g_marks[device]), 2 * kMarkBlocks * 3 * sizeof(unsigned long long)) !=
          hipSuccess)
    rc = -3;
  if (!rc) {
    hipLaunchKernelGGL(clock_mark_kernel, dim3(kMarkBlocks), dim3(64), 0, static_cast<hipStream_t>(stream),
                       g_marks[device] + which * kMarkBlocks * 3);
    rc = hipGetLastError() == hipSuccess ? 0 : -4;
  }
  (void)hipSetDevice(prev);
  return rc;
}

// After the end mark has run (the caller synchronized the stream): the median clock over the CUs
// seen in both marks (MHz), the realtime between the marks (s), and the number of CUs matched.
int clockprobe_read(int device, double* mhz, double* seconds, int* units) {
  if (device < 0 || device >= 64 || !g_marks[device]) return -1;
  static unsigned long long h[2][kMarkBlocks][3];
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) return -2;
  const bool ok = hipMemcpy(h, g_marks[device], sizeof h, hipMemcpyDeviceToHost) == hipSuccess;
  (void)hipSetDevice(prev);
  if (!ok) return -3;
  std::map<unsigned long long, int> first_end;
  for (int k = kMarkBlocks; k-- > 0;) first_end[h[1][k][0]] = k;
  std::map<unsigned long long, int> seen;
  std::vector<double> rates;
  double secs = 0;
  for (int k = 0; k < kMarkBlocks; ++k) {
    const unsigned long long key = h[0][k][0];
    auto e = first_end.find(key);
    if (e == first_end.end() || seen.count(key)) continue;
    seen[key] = 1;
    const unsigned long long* a = h[0][k];
    const unsigned long long* b = h[1][e->second];
    if (b[2] <= a[2] || b[1] <= a[1]) continue;
    const double dr = (double)(b[2] - a[2]);
    rates.push_back(100.0 * (double)(b[1] - a[1]) / dr);
    secs += dr / 1e8;
  }
  if (rates.empty()) return -4;
  std::sort(rates.begin(), rates.end());
  *mhz = rates[rates.size() / 2];
  *seconds = secs / (double)rates.size();
  *units = (int)rates.size();
  return 0;
}

// The device's PCI address ("0000:05:00.0"), to find it among amdsmi's processors.
int clockprobe_pci_bus_id(int device, char* buf, int len) {
  return hipDeviceGetPCIBusId(buf, len, device) == hipSuccess ? 0 : -1;
}

}  // extern "C"
