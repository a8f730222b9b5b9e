// Diagnostic: the shader clock over time, sampled by one wave on its own stream while other work
// runs. Sample i = (s_memtime, s_memrealtime) after ~`sleep_units` x 64 x 127 idle cycles; the
// clock between samples is d(memtime) / d(memrealtime) x 100 MHz (MI355X_MICROARCH.md, DVFS).
// The wave exits after n samples. Build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC
// clockprobe.hip -o libclockprobe.so (tools/clock_probe.py loads it).
#include <hip/hip_runtime.h>

__global__ void k_clock_probe(unsigned long long* out, int n, int sleep_units) {
  for (int i = 0; i < n; ++i) {
    const unsigned long long c = __builtin_amdgcn_s_memtime();
    const unsigned long long w = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (threadIdx.x == 0) {
      out[2 * i] = c;
      out[2 * i + 1] = w;
    }
    for (int k = 0; k < sleep_units; ++k) __builtin_amdgcn_s_sleep(127);
  }
}

extern "C" int clock_probe_launch(void* stream, unsigned long long* out, int n, int sleep_units) {
  hipLaunchKernelGGL(k_clock_probe, dim3(1), dim3(64), 0, (hipStream_t)stream, out, n, sleep_units);
  return (int)hipGetLastError();
}
