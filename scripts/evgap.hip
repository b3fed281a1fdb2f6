// Cross-stream fork cost on the producer stream (companion of scripts/diag_event_gap.py):
//   plain      k1; k2                                              (same stream)
//   marker     k1; hipEventRecord(ev); side waits ev; k2           (a barrier/marker packet on the producer)
//   bound      hipExtLaunchKernelGGL(k1, stop = ev); side waits ev; k2   (the event rides on k1's packet)
//   rec_only   k1; hipEventRecord(ev); k2                          (no consumer)
//   side_only  k1; independent small kernel on the side stream; k2 (no event)
//   rec_wait   k1; hipEventRecord(ev); side waits ev; k2           (no side kernel)
//   wait_done  k1; wait on an event of the side stream completed long ago; k2   (consumer side)
//   wake       side: long kernel + record; main: short kernel, wait, k2: k2's start minus the side
//              kernel's end is the wake-up latency of an unsatisfied cross-queue wait
// Build: hipcc --offload-arch=gfx950 -O2 scripts/evgap.hip -o scripts/evgap
// Run:   rocprofv3 --kernel-trace --output-format csv -d gpurun_out/evgap2 -- scripts/evgap
//        python scripts/diag_event_gap.py --analyze-bin <kernel_trace.csv>
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <unistd.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__global__ void big_pass(float4* __restrict__ p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    float4 v = p[i];
    v.x += 1.f; v.y += 1.f; v.z += 1.f; v.w += 1.f;
    p[i] = v;
  }
}

__global__ void small_pass(float* __restrict__ p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1.f;
}

int main() {
  const int n4 = 4 << 20;  // 64 MB
  float4* big = nullptr;
  float* small = nullptr;
  CK(hipMalloc(&big, (size_t)n4 * sizeof(float4)));
  CK(hipMalloc(&small, 65536 * sizeof(float)));
  CK(hipMemset(big, 0, (size_t)n4 * sizeof(float4)));
  CK(hipMemset(small, 0, 65536 * sizeof(float)));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const dim3 g(2048), b(256);
  hipEvent_t done_ev;
  CK(hipEventCreateWithFlags(&done_ev, hipEventDisableTiming));
  for (int phase = 0; phase < 6; ++phase) {
    for (int r = 0; r < 40; ++r) {
      if (phase == 2) {
        hipExtLaunchKernelGGL(big_pass, g, b, 0, s0, nullptr, ev, 0, big, n4);
      } else {
        hipLaunchKernelGGL(big_pass, g, b, 0, s0, big, n4);
        if (phase == 1 || phase == 3 || phase == 5) CK(hipEventRecord(ev, s0));
      }
      if (phase == 1 || phase == 2 || phase == 5) CK(hipStreamWaitEvent(s1, ev, 0));
      if (phase == 1 || phase == 2 || phase == 4)
        hipLaunchKernelGGL(small_pass, dim3(256), dim3(256), 0, s1, small, 65536);
      hipLaunchKernelGGL(big_pass, g, b, 0, s0, big, n4);
    }
    CK(hipDeviceSynchronize());
    usleep(20000);
  }
  // wait_done
  hipLaunchKernelGGL(small_pass, dim3(256), dim3(256), 0, s1, small, 65536);
  CK(hipEventRecord(done_ev, s1));
  CK(hipDeviceSynchronize());
  for (int r = 0; r < 40; ++r) {
    hipLaunchKernelGGL(big_pass, g, b, 0, s0, big, n4);
    CK(hipStreamWaitEvent(s0, done_ev, 0));
    hipLaunchKernelGGL(big_pass, g, b, 0, s0, big, n4);
  }
  CK(hipDeviceSynchronize());
  usleep(20000);
  // wake: the side stream's 8 passes end well after the main stream's short kernel
  for (int r = 0; r < 40; ++r) {
    for (int q = 0; q < 8; ++q) hipLaunchKernelGGL(big_pass, g, b, 0, s1, big + (size_t)n4 / 2, n4 / 2);
    CK(hipEventRecord(ev, s1));
    hipLaunchKernelGGL(small_pass, dim3(256), dim3(256), 0, s0, small, 65536);
    CK(hipStreamWaitEvent(s0, ev, 0));
    hipLaunchKernelGGL(big_pass, g, b, 0, s0, big, n4 / 2);
    CK(hipDeviceSynchronize());
  }
  CK(hipGetLastError());
  std::printf("ok\n");
  return 0;
}
