#pragma once
// In-kernel clock stamps for diagnostic builds only (-DPNTF_CLOCK_STAMP; tests/diag/
// clock_probe.py): the effective shader clock of a launch is Δs_memtime / Δs_memrealtime ×
// 100 MHz per workgroup (MI355X_MICROARCH.md, 'DVFS give-back' item 6).  Workgroup b's lane 0
// writes (Δmemtime, Δrealtime) of its lifetime to pntf_clock_stamps[2b..2b+1] with a vector
// store; no output is computed from them.  In the shipped library PNTF_CLOCK_SCOPE is empty.
#ifdef PNTF_CLOCK_STAMP
__device__ unsigned long long pntf_clock_stamps[2 * 8192];
struct PntfStamp {
  unsigned long long t0, r0;
  __device__ PntfStamp() : t0(__builtin_amdgcn_s_memtime()), r0(__builtin_amdgcn_s_memrealtime()) {}
  __device__ ~PntfStamp() {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x < 8192) {
      pntf_clock_stamps[2 * blockIdx.x] = t1 - t0;
      pntf_clock_stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
  }
};
#define PNTF_CLOCK_SCOPE PntfStamp pntf_stamp_
extern "C" __attribute__((weak)) int pntf_diag_clock_stamps(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pntf_clock_stamps),
                                  sizeof(unsigned long long) * 2 * (n < 8192 ? n : 8192), 0,
                                  hipMemcpyDeviceToHost);
}
#else
#define PNTF_CLOCK_SCOPE \
  do {         \
  } while (0)
#endif
