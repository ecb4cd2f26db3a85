// Node topology probe: which local GPU pairs are joined by a direct xGMI link.
//
// The schedules of mp4x assume the MI355X node shape — 8 GPUs, every pair one xGMI hop apart
// (7 links per GPU), peer memory readable by kernels.  The reference has no counterpart (its
// topology is "hosts on 1 GbE", README.md:300); here the probe is evidence that a multi-GPU run
// really crossed xGMI (bench.py records it), and the device engine logs a warning when a pair is
// not a single xGMI hop (PCIe-only boxes still work: the autotuners choose from measurements).
#include <hip/hip_runtime.h>

#include <cstdint>

// For every ordered pair (a, b) of the n visible devices fill row-major n*n arrays:
//   link[a*n+b]   HSA link type (4 = xGMI, 2 = PCIe; -1 = unknown / a == b)
//   hops[a*n+b]   hop count (0 on the diagonal)
//   access[a*n+b] hipDevP2PAttrAccessSupported
//   rank[a*n+b]   hipDevP2PAttrPerformanceRank
//   atomics[a*n+b] hipDevP2PAttrNativeAtomicSupported
// Returns the number of devices written (<= cap), or -(hipError) on failure.  Touches no
// device memory; safe to call before any allocation.
extern "C" int mp4x_topology(int cap, int* link, int* hops, int* access, int* rank, int* atomics) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) return -(int)e;
  if (n > cap) n = cap;
  for (int a = 0; a < n; ++a) {
    for (int b = 0; b < n; ++b) {
      const int i = a * n + b;
      link[i] = -1;
      hops[i] = 0;
      access[i] = a == b;
      rank[i] = 0;
      atomics[i] = a == b;
      if (a == b) continue;
      uint32_t lt = 0, hc = 0;
      if (hipExtGetLinkTypeAndHopCount(a, b, &lt, &hc) == hipSuccess) {
        link[i] = (int)lt;
        hops[i] = (int)hc;
      }
      int v = 0;
      if (hipDeviceGetP2PAttribute(&v, hipDevP2PAttrAccessSupported, a, b) == hipSuccess) access[i] = v;
      if (hipDeviceGetP2PAttribute(&v, hipDevP2PAttrPerformanceRank, a, b) == hipSuccess) rank[i] = v;
      if (hipDeviceGetP2PAttribute(&v, hipDevP2PAttrNativeAtomicSupported, a, b) == hipSuccess) atomics[i] = v;
    }
  }
  (void)hipGetLastError();   // a failed query must not poison the next kernel launch's error check
  return n;
}
