// Microbenchmark: the cost of the work-queue tickets the ETA / GCM kernels
// draw (one device-scope atomicAdd on one global counter per unit, its value
// waited on by the wave).  Empty units, so the kernel time is the queue's:
//   mode 0: one counter, a ticket per wave-unit (the ETA kernel's queue)
//   mode 1: eight counters, workgroup g draws from counter g % 8 (one per XCD)
//   mode 2: one counter, a ticket for 4 units at a time
// Prints one JSON line per (mode, units, waves per workgroup).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(768) void queue_kernel(unsigned *q, unsigned units, int mode, unsigned *sink) {
  const int lane = threadIdx.x & 63;
  unsigned acc = 0;
  unsigned *ctr = mode == 1 ? q + 64 * (blockIdx.x & 7) : q;
  const unsigned per = mode == 1 ? (units + 7) / 8 : units;
  const unsigned step = mode == 2 ? 4u : 1u;
  for (;;) {
    unsigned t = 0;
    if (lane == 0) t = atomicAdd(ctr, step);
    t = __builtin_amdgcn_readfirstlane(t);
    if (t >= per) break;
    acc += t + lane;
  }
  if (acc == 0xdeadbeef) sink[0] = acc;
}

int main() {
  unsigned *q, *sink;
  hipMalloc(&q, 8 * 64 * 4);
  hipMalloc(&sink, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 3; ++mode)
    for (unsigned units : {4096u, 16384u, 65536u}) {
      float best = 1e9f;
      for (int rep = 0; rep < 5; ++rep) {
        hipMemset(q, 0, 8 * 64 * 4);
        hipEventRecord(e0);
        hipLaunchKernelGGL(queue_kernel, dim3(256), dim3(768), 0, 0, q, units, mode, sink);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      printf("{\"mode\": %d, \"units\": %u, \"ms\": %.4f, \"ns_per_ticket\": %.2f}\n", mode, units, best,
             best * 1e6 / (mode == 2 ? units / 4.0 : units));
    }
  return 0;
}
