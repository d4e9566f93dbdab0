// Diagnostic (not a test, not product code): host-side cost of the HIP calls
// the copying to_tensor_fn path makes per batch, on idle and busy streams:
// hipMemcpyAsync H2D from pinned memory (1 MB / 17 MB), the same from several
// threads at once on one stream, hipEventRecord, cross-stream
// hipStreamWaitEvent, a kernel launch, and a copy stream + event handoff.
// build: hipcc -O2 --offload-arch=gfx950 tools/probes/hip_api_cost.cpp -o tools/probes/hip_api_cost -lpthread
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>
#include <thread>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void k_spin(long long cycles, int *sink) {
  long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && sink) sink[blockIdx.x] = 1;
}

__global__ void k_nop(int *p) {
  if (p && threadIdx.x == 0) p[blockIdx.x] = 0;
}

int main() {
  const size_t N = 17 << 20, MB = 1 << 20;
  void *h, *d, *d2;
  int *sink;
  CK(hipHostMalloc(&h, N, hipHostMallocDefault));
  CK(hipMalloc(&d, N));
  CK(hipMalloc(&d2, N));
  CK(hipMalloc((void **)&sink, 1 << 20));
  hipStream_t s[5];
  for (auto &x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  hipEvent_t ev[64];
  for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // ~2 ms of spin on 1 workgroup (clock64 ~100 MHz constant? measured below)
  k_spin<<<1, 64, 0, s[0]>>>(1000, sink);
  CK(hipDeviceSynchronize());
  const int R = 40;
  auto busy = [&](hipStream_t st) { k_spin<<<256, 64, 0, st>>>(2000000, sink); };

  for (int b = 0; b < 2; ++b) {
    const char *tag = b ? "busy" : "idle";
    double t = 0;
    for (int r = 0; r < R; ++r) {
      if (b) busy(s[1]);
      double a = now_us();
      CK(hipMemcpyAsync(d, h, MB, hipMemcpyHostToDevice, s[1]));
      t += now_us() - a;
      CK(hipStreamSynchronize(s[1]));
    }
    printf("hipMemcpyAsync 1MB (%s stream): %.1f us\n", tag, t / R);
    t = 0;
    for (int r = 0; r < R; ++r) {
      if (b) busy(s[1]);
      double a = now_us();
      CK(hipMemcpyAsync(d, h, N, hipMemcpyHostToDevice, s[1]));
      t += now_us() - a;
      CK(hipStreamSynchronize(s[1]));
    }
    printf("hipMemcpyAsync 17MB (%s stream): %.1f us\n", tag, t / R);
    t = 0;
    for (int r = 0; r < R; ++r) {
      if (b) busy(s[1]);
      double a = now_us();
      for (int k = 0; k < 17; ++k)
        CK(hipMemcpyAsync((char *)d + k * MB, (char *)h + k * MB, MB, hipMemcpyHostToDevice, s[1]));
      t += now_us() - a;
      CK(hipStreamSynchronize(s[1]));
    }
    printf("17 x hipMemcpyAsync 1MB, one thread (%s stream): %.1f us total\n", tag, t / R);
    t = 0;
    for (int r = 0; r < R; ++r) {
      if (b) busy(s[1]);
      double a = now_us();
      std::vector<std::thread> th;
      for (int q = 0; q < 6; ++q)
        th.emplace_back([&, q] {
          for (int k = q; k < 17; k += 6)
            (void)hipMemcpyAsync((char *)d + k * MB, (char *)h + k * MB, MB, hipMemcpyHostToDevice, s[1]);
        });
      for (auto &x : th) x.join();
      t += now_us() - a;
      CK(hipStreamSynchronize(s[1]));
    }
    printf("17 x hipMemcpyAsync 1MB from 6 threads (%s stream): %.1f us total (incl. thread start)\n", tag, t / R);
    t = 0;
    double tw = 0, tl = 0;
    for (int r = 0; r < R; ++r) {
      if (b) busy(s[1]);
      double a = now_us();
      CK(hipEventRecord(ev[r % 64], s[1]));
      double m = now_us();
      CK(hipStreamWaitEvent(s[2], ev[r % 64], 0));
      double m2 = now_us();
      k_nop<<<1, 64, 0, s[2]>>>(sink);
      double e = now_us();
      t += m - a;
      tw += m2 - m;
      tl += e - m2;
      CK(hipDeviceSynchronize());
    }
    printf("hipEventRecord %.1f us, hipStreamWaitEvent (cross-stream) %.1f us, launch after wait %.1f us (%s)\n",
           t / R, tw / R, tl / R, tag);
    t = 0;
    for (int r = 0; r < R; ++r) {
      if (b) busy(s[1]);
      double a = now_us();
      for (int k = 0; k < 8; ++k) k_nop<<<256, 256, 0, s[1]>>>(sink);
      t += now_us() - a;
      CK(hipDeviceSynchronize());
    }
    printf("8 kernel launches (%s stream): %.1f us total\n", tag, t / R);
    // copy-stream handoff as a pipeline would do it: DMA on s[4], record, the
    // compute stream waits, kernel, record kernel-done, copy stream waits on it
    t = 0;
    for (int r = 0; r < R; ++r) {
      if (b) {
        busy(s[1]);
        busy(s[2]);
        busy(s[3]);
      }
      hipStream_t cs = s[1 + r % 3];
      double a = now_us();
      CK(hipStreamWaitEvent(s[4], ev[(r + 63) % 64], 0));
      CK(hipMemcpyAsync(d, h, N, hipMemcpyHostToDevice, s[4]));
      CK(hipEventRecord(ev[r % 64], s[4]));
      CK(hipStreamWaitEvent(cs, ev[r % 64], 0));
      for (int k = 0; k < 6; ++k) k_nop<<<256, 256, 0, cs>>>(sink);
      CK(hipEventRecord(ev[(r + 32) % 64], cs));
      t += now_us() - a;
      if (r % 3 == 2) CK(hipDeviceSynchronize());
    }
    CK(hipDeviceSynchronize());
    printf("copy-stream handoff (wait, 17MB DMA, record, wait, 6 launches, record) (%s): %.1f us\n", tag, t / R);
  }
  // a small H2D copy (the plan blob, 100 KB) enqueued on a stream that waits
  // for an event of a copy stream still busy with a 17 MB DMA: does the
  // enqueue block the host until the event fires?
  for (size_t small : {(size_t)4 << 10, (size_t)100 << 10, (size_t)1 << 20}) {
    double t = 0, tw = 0;
    for (int r = 0; r < 10; ++r) {
      CK(hipMemcpyAsync(d2, h, N, hipMemcpyHostToDevice, s[4]));
      CK(hipEventRecord(ev[r % 64], s[4]));
      CK(hipStreamWaitEvent(s[1], ev[r % 64], 0));
      double a = now_us();
      CK(hipMemcpyAsync(d, h, small, hipMemcpyHostToDevice, s[1]));
      double b = now_us();
      k_nop<<<1, 64, 0, s[1]>>>(sink);
      double c = now_us();
      t += b - a;
      tw += c - b;
      CK(hipDeviceSynchronize());
    }
    printf("H2D %zu KB on a stream waiting for a busy copy stream: enqueue %.1f us, next launch %.1f us\n",
           small >> 10, t / 10, tw / 10);
  }
  // how long a 17MB DMA takes while 3 streams run kernels
  {
    hipEvent_t a, z;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&z));
    busy(s[1]);
    busy(s[2]);
    CK(hipEventRecord(a, s[4]));
    CK(hipMemcpyAsync(d, h, N, hipMemcpyHostToDevice, s[4]));
    CK(hipEventRecord(z, s[4]));
    CK(hipDeviceSynchronize());
    float ms;
    CK(hipEventElapsedTime(&ms, a, z));
    printf("17MB DMA on a copy stream while 2 streams spin: %.1f us\n", ms * 1e3);
  }
  printf("done\n");
  return 0;
}
