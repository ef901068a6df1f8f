// clockprobe.hip -- the effective engine clock over a timed region, read on the GPU itself
// (bench.py's `clock` objects; measurement infrastructure, not part of libefeshash).
//
// Two tiny marker launches on the measured stream bracket the region: each of their workgroups
// (one wave, at least one lands on every XCD) records its XCD (HW_REG_XCC_ID), s_memtime and
// s_memrealtime (the 100 MHz constant clock).  s_memtime counts per XCD, so the start and end
// marks are matched by XCD: the memtime ticks between them over the realtime between them is the
// clock the XCD ran at meanwhile.  The marks are ordinary kernels in stream order -- nothing runs
// beside the measured work, nothing waits on the host.  Calibration against GRBM_GUI_ACTIVE and
// amdsmi: profiles/r05_clock/.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kMarkBlocks = 64;  // dealt round-robin over the 8 XCDs

__global__ void clock_mark_kernel(unsigned long long* out) {
  if (threadIdx.x != 0) return;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  const unsigned long long r = __builtin_amdgcn_s_memrealtime();
  unsigned long long* o = out + 3 * blockIdx.x;
  o[0] = xcc & 0xfu;
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

// After the end mark has run (the caller synchronized the stream): the mean clock over the XCDs
// seen in both marks (MHz), the realtime between the marks (s), and the XCDs matched.
int clockprobe_read(int device, double* mhz, double* seconds, int* xcds) {
  if (device < 0 || device >= 64 || !g_marks[device]) return -1;
  unsigned long long h[2][kMarkBlocks][3];
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) return -2;
  const bool ok = hipMemcpy(h, g_marks[device], sizeof h, hipMemcpyDeviceToHost) == hipSuccess;
  (void)hipSetDevice(prev);
  if (!ok) return -3;
  double sum = 0, secs = 0;
  int n = 0;
  for (unsigned x = 0; x < 16; ++x) {
    int a = -1, b = -1;
    for (int k = 0; k < kMarkBlocks; ++k) {
      if (a < 0 && h[0][k][0] == x) a = k;
      if (b < 0 && h[1][k][0] == x) b = k;
    }
    if (a < 0 || b < 0 || h[1][b][2] <= h[0][a][2]) continue;
    const double dr = (double)(h[1][b][2] - h[0][a][2]);
    sum += 100.0 * (double)(h[1][b][1] - h[0][a][1]) / dr;
    secs += dr / 1e8;
    ++n;
  }
  if (!n) return -4;
  *mhz = sum / n;
  *seconds = secs / n;
  *xcds = n;
  return 0;
}

// The device's PCI address ("0000:05:00.0"), to find it among amdsmi's processors.
int clockprobe_pci_bus_id(int device, char* buf, int len) {
  return hipDeviceGetPCIBusId(buf, len, device) == hipSuccess ? 0 : -1;
}

}  // extern "C"
