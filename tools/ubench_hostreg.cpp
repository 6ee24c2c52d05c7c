// tools/ubench_hostreg.cpp -- what does it cost to pin an uploader's pageable buffers instead
// of copying them into pinned staging?  512 MiB: malloc'd (touched) and a file mmap'd
// (MAP_PRIVATE, pre-faulted); hipHostRegister / hipHostUnregister time, then the H2D rate from
// the registered range vs a pinned hipHostMalloc buffer vs plain pageable memory.
//   hipcc -O2 -o tools/ubench_hostreg tools/ubench_hostreg.cpp
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double h2d(void* dev, const void* src, size_t n) {
  (void)hipMemcpy(dev, src, n, hipMemcpyHostToDevice);  // warm
  const double t0 = now();
  for (int i = 0; i < 3; ++i) (void)hipMemcpy(dev, src, n, hipMemcpyHostToDevice);
  return 3.0 * n / (now() - t0) / 1e9;
}

int main() {
  const size_t N = 512ull << 20;
  void* dev = nullptr;
  if (hipMalloc(&dev, N) != hipSuccess) { std::printf("no device\n"); return 1; }
  // pinned reference
  void* pin = nullptr;
  double t0 = now();
  (void)hipHostMalloc(&pin, N, hipHostMallocDefault);
  const double t_pin = now() - t0;
  std::memset(pin, 1, N);
  std::printf("hipHostMalloc 512 MiB: %.2f ms; H2D from it %.1f GB/s\n", 1e3 * t_pin, h2d(dev, pin, N));
  // malloc'd, touched
  char* m = static_cast<char*>(std::malloc(N));
  std::memset(m, 2, N);
  std::printf("pageable malloc H2D %.1f GB/s\n", h2d(dev, m, N));
  for (int rep = 0; rep < 3; ++rep) {
    t0 = now();
    hipError_t e = hipHostRegister(m, N, hipHostRegisterDefault);
    const double t_reg = now() - t0;
    double rate = e == hipSuccess ? h2d(dev, m, N) : 0;
    t0 = now();
    hipError_t u = e == hipSuccess ? hipHostUnregister(m) : hipSuccess;
    std::printf("malloc 512 MiB: hipHostRegister %s %.2f ms, H2D %.1f GB/s, unregister %s %.2f ms\n",
                hipGetErrorString(e), 1e3 * t_reg, rate, hipGetErrorString(u), 1e3 * (now() - t0));
  }
  // file mmap (MAP_PRIVATE, read-only), pre-faulted
  const char* path = "/tmp/s3h_hostreg.bin";
  FILE* f = std::fopen(path, "wb");
  for (size_t off = 0; off < N; off += 1 << 20) std::fwrite(m + off, 1, 1 << 20, f);
  std::fclose(f);
  const int fd = open(path, O_RDONLY);
  char* fm = static_cast<char*>(mmap(nullptr, N, PROT_READ, MAP_PRIVATE, fd, 0));
  volatile char sink = 0;
  for (size_t off = 0; off < N; off += 4096) sink ^= fm[off];
  std::printf("file mmap pageable H2D %.1f GB/s\n", h2d(dev, fm, N));
  for (unsigned flags : {unsigned(hipHostRegisterDefault), unsigned(hipHostRegisterReadOnly)}) {
    t0 = now();
    hipError_t e = hipHostRegister(fm, N, flags);
    const double t_reg = now() - t0;
    if (e != hipSuccess) (void)hipGetLastError();
    double rate = e == hipSuccess ? h2d(dev, fm, N) : 0;
    t0 = now();
    hipError_t u = e == hipSuccess ? hipHostUnregister(fm) : hipSuccess;
    std::printf("file mmap 512 MiB flags=%u: hipHostRegister %s %.2f ms, H2D %.1f GB/s, unregister %.2f ms\n",
                flags, hipGetErrorString(e), 1e3 * t_reg, rate, 1e3 * (now() - t0));
  }
  munmap(fm, N);
  close(fd);
  std::remove(path);
  // memcpy rate into pinned memory with 1 thread (the staging cost per byte)
  t0 = now();
  std::memcpy(pin, m, N);
  std::printf("memcpy pageable->pinned 1 thread: %.1f GB/s\n", N / (now() - t0) / 1e9);
  std::free(m);
  (void)hipHostFree(pin);
  (void)hipFree(dev);
  return sink == 42 ? 1 : 0;
}
