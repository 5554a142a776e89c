// Probe (tool): cost of DMA'ing a page-cache file to the GPU by registering its mmap
// (hipHostRegister, no CPU copy) against pread into a page-locked buffer + H2D.
//   ./hostreg_probe FILE   (FILE already in the page cache)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>
static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
int main(int argc, char **argv) {
  int fd = open(argv[1], O_RDONLY);
  struct stat st;
  fstat(fd, &st);
  size_t len = st.st_size & ~(size_t)4095;
  void *dev;
  CK(hipMalloc(&dev, len));
  for (int rep = 0; rep < 3; rep++) {
    double t0 = now();
    void *p = mmap(nullptr, len, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
    double t1 = now();
    hipError_t e = hipHostRegister(p, len, hipHostRegisterReadOnly);
    double t2 = now();
    if (e != hipSuccess) { printf("register: %s\n", hipGetErrorString(e)); return 1; }
    CK(hipMemcpy(dev, p, len, hipMemcpyHostToDevice));
    double t3 = now();
    CK(hipHostUnregister(p));
    munmap(p, len);
    double t4 = now();
    printf("mmap %.4f register %.4f h2d %.4f (%.1f GB/s) unregister+munmap %.4f total %.4f s\n", t1 - t0, t2 - t1,
           t3 - t2, len / (t3 - t2) / 1e9, t4 - t3, t4 - t0);
  }
  void *pin;
  CK(hipHostMalloc(&pin, len, hipHostMallocDefault));
  for (int rep = 0; rep < 3; rep++) {
    double t0 = now();
    const int nt = 4;
    std::vector<std::thread> th;
    for (int k = 0; k < nt; k++)
      th.emplace_back([&, k] {
        size_t a = len / nt * k, b = k == nt - 1 ? len : len / nt * (k + 1);
        while (a < b) {
          ssize_t r = pread(fd, (char *)pin + a, b - a, a);
          if (r <= 0) break;
          a += r;
        }
      });
    for (auto &t : th) t.join();
    double t1 = now();
    CK(hipMemcpy(dev, pin, len, hipMemcpyHostToDevice));
    double t2 = now();
    printf("pread(4 threads) %.4f (%.1f GB/s) h2d %.4f (%.1f GB/s) total %.4f s\n", t1 - t0, len / (t1 - t0) / 1e9,
           t2 - t1, len / (t2 - t1) / 1e9, t2 - t0);
  }
  return 0;
}
