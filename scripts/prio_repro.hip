// Minimal two-stream repro for the "high-priority stream + cross-stream hand-offs" slowdown
// (profiles/r3z_priority_vs_sync.md).
//
// A chain of small kernels on stream A (the critical path); every PERIOD kernels stream B (the
// comm stream) takes a hand-off from A, runs one small kernel, and hands back to A -- the
// reducer's pattern (bucket launch waits for compute; finalize waits for comm).  Modes:
//   A priority: high / normal;  B priority: normal / high;
//   hand-off primitive: none (B idle), hipEvent (record + wait), or stream memory ops
//   (hipStreamWriteValue64 on the producer, hipStreamWaitValue64 on the consumer).
// Prints us per A-kernel for each combination (median of REPS, one process).
//
//   hipcc --offload-arch=gfx950 -O2 scripts/prio_repro.hip -o build/prio_repro && ./build/prio_repro
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

__global__ void small_kernel(float* p, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float v = p[i];
  for (int k = 0; k < iters; ++k) v = v * 0.999f + 0.001f;
  p[i] = v;
}

enum Sync { NONE = 0, EVENT = 1, VALUE = 2, ONEWAY = 3 };
// ONEWAY: the reducer's pattern during backward -- A records an event every PERIOD kernels, B
// waits for it and runs its kernel, but A never waits for B (until the end of the run)

int main(int argc, char** argv) {
  const int nk = argc > 1 ? atoi(argv[1]) : 400;      // kernels on stream A per run
  const int period = argc > 2 ? atoi(argv[2]) : 20;   // hand-off every `period` A kernels
  const int reps = argc > 3 ? atoi(argv[3]) : 7;
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));  // lo = least (normal), hi = greatest
  float *bufA, *bufB;
  CK(hipMalloc(&bufA, 256 * 256 * sizeof(float)));
  CK(hipMalloc(&bufB, 256 * 256 * sizeof(float)));
  CK(hipMemset(bufA, 0, 256 * 256 * sizeof(float)));
  CK(hipMemset(bufB, 0, 256 * 256 * sizeof(float)));
  // [0]: A -> B sequence, [1]: B -> A sequence; signal memory is allocated one 8-byte word at a
  // time (hipMallocSignalMemory refuses larger sizes on MI355X / ROCm 7.2)
  uint64_t* fl[2] = {nullptr, nullptr};
  for (int i = 0; i < 2; ++i) {
    CK(hipExtMallocWithFlags((void**)&fl[i], sizeof(uint64_t), hipMallocSignalMemory));
    CK(hipMemset(fl[i], 0, sizeof(uint64_t)));
  }
  int wv = 0;
  CK(hipDeviceGetAttribute(&wv, hipDeviceAttributeCanUseStreamWaitValue, 0));
  printf("priority range least %d greatest %d; stream wait value supported: %d\n", lo, hi, wv);
  printf("%-8s %-8s %-6s %10s %10s\n", "A_prio", "B_prio", "sync", "us/kernel", "min");
  const char* sname[] = {"none", "event", "value", "oneway"};
  uint64_t seq = 0;
  for (int pa = 0; pa < 2; ++pa)
    for (int pb = 0; pb < 2; ++pb)
      for (int sy = 0; sy < 4; ++sy) {
        if (sy == VALUE && !wv) continue;
        hipStream_t A, B;
        CK(hipStreamCreateWithPriority(&A, hipStreamNonBlocking, pa ? hi : lo));
        CK(hipStreamCreateWithPriority(&B, hipStreamNonBlocking, pb ? hi : lo));
        hipEvent_t e0, e1, ea, eb;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventCreateWithFlags(&ea, hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
        std::vector<float> t;
        for (int r = 0; r < reps + 1; ++r) {
          CK(hipDeviceSynchronize());
          CK(hipEventRecord(e0, A));
          for (int k = 0; k < nk; ++k) {
            hipLaunchKernelGGL(small_kernel, dim3(256), dim3(256), 0, A, bufA, 200);
            if (sy != NONE && (k + 1) % period == 0) {
              ++seq;
              if (sy == EVENT || sy == ONEWAY) {
                CK(hipEventRecord(ea, A));
                CK(hipStreamWaitEvent(B, ea, 0));
              } else {
                CK(hipStreamWriteValue64(A, fl[0], seq, 0));
                CK(hipStreamWaitValue64(B, fl[0], seq, hipStreamWaitValueGte, ~0ull));
              }
              hipLaunchKernelGGL(small_kernel, dim3(64), dim3(256), 0, B, bufB, 100);
              if (sy == ONEWAY) {
              } else if (sy == EVENT) {
                CK(hipEventRecord(eb, B));
                CK(hipStreamWaitEvent(A, eb, 0));
              } else {
                CK(hipStreamWriteValue64(B, fl[1], seq, 0));
                CK(hipStreamWaitValue64(A, fl[1], seq, hipStreamWaitValueGte, ~0ull));
              }
            }
          }
          if (sy == ONEWAY) {  // join B once at the end
            CK(hipEventRecord(eb, B));
            CK(hipStreamWaitEvent(A, eb, 0));
          }
          CK(hipEventRecord(e1, A));
          CK(hipEventSynchronize(e1));
          float ms = 0.f;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (r > 0) t.push_back(ms * 1000.f / nk);
        }
        std::sort(t.begin(), t.end());
        printf("%-8s %-8s %-6s %10.2f %10.2f\n", pa ? "high" : "normal", pb ? "high" : "normal", sname[sy],
               t[t.size() / 2], t[0]);
        fflush(stdout);
        CK(hipStreamSynchronize(A));
        CK(hipStreamSynchronize(B));
        CK(hipEventDestroy(e0));
        CK(hipEventDestroy(e1));
        CK(hipEventDestroy(ea));
        CK(hipEventDestroy(eb));
        CK(hipStreamDestroy(A));
        CK(hipStreamDestroy(B));
      }
  CK(hipFree(bufA));
  CK(hipFree(bufB));
  CK(hipFree(fl[0]));
  CK(hipFree(fl[1]));
  return 0;
}
