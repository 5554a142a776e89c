// Node input probe: what a node's host can feed N GPU workers from
// page-cache segments, with no GPU call at all.
//
// Each pipeline is one process, like one `-H gpu:N` worker (fd.py:130: the segment file on the
// worker's stdin; worker.py Source._read_mkv_pread): T threads positional-read (pread) the
// segment's bytes from the page cache into one of three locked "batch" buffers of B bytes
// (worker.py's page-locked batches; mlock here, hipHostMalloc in the worker), and, with
// --dma, one more thread reads every filled batch once before it is refilled (a stand-in for the
// GPU's DMA read of the batch over PCIe: the same DRAM read traffic, done by a CPU).  Pipeline
// p binds to NUMA node (p * nodes / P) as worker.bind_numa binds a worker to its GPU's node
// (CPUs of the node that are allowed, and MPOL_PREFERRED memory).
//
// Output: one JSON line: per pipeline and aggregate GB/s of segment input, the implied 4K
// frames/s (12,441,600 bytes per yuv420p frame), CPU seconds per GB, and the host's CPU quota.
//
// build: gcc -O2 -pthread -o node_input_probe tools/node_input_probe.c
// usage: node_input_probe [--pipelines P] [--threads T] [--segment-mb M] [--batch-mb B]
//                         [--seconds S] [--dma] [--dir DIR]
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

static int P = 8, T = 4, DMA = 0;
static size_t SEG = (size_t)120 * 12441600, BATCH = (size_t)256 << 20;
static double SECONDS = 10.0;
static const char *DIR_ = "/tmp";

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int nnodes(void) {
  int n = 0;
  char p[64];
  for (;; n++) {
    snprintf(p, sizeof p, "/sys/devices/system/node/node%d/cpulist", n);
    if (access(p, R_OK)) break;
  }
  return n ? n : 1;
}

static void bind_node(int node) {
  char p[80], buf[4096];
  snprintf(p, sizeof p, "/sys/devices/system/node/node%d/cpulist", node);
  FILE *f = fopen(p, "r");
  if (!f) return;
  if (!fgets(buf, sizeof buf, f)) buf[0] = 0;
  fclose(f);
  cpu_set_t allowed, want;
  CPU_ZERO(&want);
  if (sched_getaffinity(0, sizeof allowed, &allowed)) return;
  for (char *s = buf; *s && *s != '\n';) {
    int a = (int)strtol(s, &s, 10), b = a;
    if (*s == '-') b = (int)strtol(s + 1, &s, 10);
    for (int c = a; c <= b && c < CPU_SETSIZE; c++)
      if (CPU_ISSET(c, &allowed)) CPU_SET(c, &want);
    if (*s == ',') s++;
  }
  if (CPU_COUNT(&want) == 0) return;
  sched_setaffinity(0, sizeof want, &want);
  unsigned long mask = 1ul << node;
  syscall(SYS_set_mempolicy, 1 /* MPOL_PREFERRED */, &mask, 64ul);
}

typedef struct {
  int fd;
  uint8_t *dst;
  size_t off, len;
} Job;

static void *pread_job(void *arg) {
  Job *j = (Job *)arg;
  size_t got = 0;
  while (got < j->len) {
    ssize_t k = pread(j->fd, j->dst + got, j->len - got, (off_t)(j->off + got));
    if (k <= 0) {
      perror("pread");
      exit(2);
    }
    got += (size_t)k;
  }
  return NULL;
}

// the DMA stand-in: reads a filled batch once (8-byte loads, summed so nothing is optimised away)
typedef struct {
  uint8_t *buf[3];
  int full[3];
  int stop;
  size_t len[3];
  pthread_mutex_t mu;
  pthread_cond_t cv;
  volatile uint64_t sink;
} Dma;

static void *dma_thread(void *arg) {
  Dma *d = (Dma *)arg;
  int i = 0;
  for (;;) {
    pthread_mutex_lock(&d->mu);
    while (!d->full[i] && !d->stop) pthread_cond_wait(&d->cv, &d->mu);
    if (!d->full[i] && d->stop) {
      pthread_mutex_unlock(&d->mu);
      return NULL;
    }
    pthread_mutex_unlock(&d->mu);
    const uint64_t *w = (const uint64_t *)d->buf[i];
    uint64_t s = 0;
    for (size_t k = 0; k < d->len[i] / 8; k++) s += w[k];
    d->sink += s;
    pthread_mutex_lock(&d->mu);
    d->full[i] = 0;
    pthread_cond_broadcast(&d->cv);
    pthread_mutex_unlock(&d->mu);
    i = (i + 1) % 3;
  }
}

static int pipeline(int p, int out_fd) {
  const int nodes = nnodes();
  const int node = (int)((long)p * nodes / P);
  bind_node(node);
  char path[512];
  snprintf(path, sizeof path, "%s/mjg_node_probe_%d_%d.seg", DIR_, (int)getppid(), p);
  int fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0600);
  if (fd < 0) {
    perror(path);
    return 2;
  }
  // the segment, written once: in the page cache as the splitter leaves it (fd.py:198-202)
  uint8_t *tmp = malloc(1 << 24);
  for (size_t i = 0; i < (1 << 24); i++) tmp[i] = (uint8_t)(i * 131 + p);
  for (size_t o = 0; o < SEG;) {
    size_t k = SEG - o < (1 << 24) ? SEG - o : (1 << 24);
    if (write(fd, tmp, k) != (ssize_t)k) {
      perror("write");
      return 2;
    }
    o += k;
  }
  free(tmp);
  fsync(fd);
  unlink(path);  // the descriptor keeps it; nothing is left behind on an early exit
  Dma d;
  memset(&d, 0, sizeof d);
  pthread_mutex_init(&d.mu, NULL);
  pthread_cond_init(&d.cv, NULL);
  for (int i = 0; i < 3; i++) {
    d.buf[i] = mmap(NULL, BATCH, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
    if (d.buf[i] == MAP_FAILED) {
      perror("mmap");
      return 2;
    }
    (void)mlock(d.buf[i], BATCH);  // page-locked when RLIMIT_MEMLOCK allows; populated either way
  }
  pthread_t dt;
  if (DMA) pthread_create(&dt, NULL, dma_thread, &d);
  // read the segment once untimed (warm page cache), then timed batches
  struct rusage r0, r1;
  double t0 = 0;
  size_t off = 0, bytes = 0;
  int i = 0, warm = 1;
  for (;;) {
    if (warm && off == 0 && bytes >= SEG) {
      warm = 0;
      bytes = 0;
      getrusage(RUSAGE_SELF, &r0);
      t0 = now();
    }
    if (!warm && now() - t0 >= SECONDS) break;
    pthread_mutex_lock(&d.mu);
    while (d.full[i]) pthread_cond_wait(&d.cv, &d.mu);
    pthread_mutex_unlock(&d.mu);
    size_t len = SEG - off < BATCH ? SEG - off : BATCH;
    pthread_t th[64];
    Job jobs[64];
    size_t part = (len + T - 1) / T;
    for (int t = 0; t < T; t++) {
      size_t a = (size_t)t * part, b = a + part < len ? a + part : len;
      jobs[t] = (Job){fd, d.buf[i] + a, off + a, b > a ? b - a : 0};
      pthread_create(&th[t], NULL, pread_job, &jobs[t]);
    }
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    bytes += len;
    off = (off + len) % SEG;
    if (DMA) {
      pthread_mutex_lock(&d.mu);
      d.full[i] = 1;
      d.len[i] = len;
      pthread_cond_broadcast(&d.cv);
      pthread_mutex_unlock(&d.mu);
    }
    i = (i + 1) % 3;
  }
  const double dt_s = now() - t0;
  if (DMA) {
    pthread_mutex_lock(&d.mu);
    d.stop = 1;
    pthread_cond_broadcast(&d.cv);
    pthread_mutex_unlock(&d.mu);
    pthread_join(dt, NULL);
  }
  getrusage(RUSAGE_SELF, &r1);
  const double cpu = (r1.ru_utime.tv_sec - r0.ru_utime.tv_sec) + (r1.ru_stime.tv_sec - r0.ru_stime.tv_sec) +
                     1e-6 * ((r1.ru_utime.tv_usec - r0.ru_utime.tv_usec) + (r1.ru_stime.tv_usec - r0.ru_stime.tv_usec));
  char line[256];
  int n = snprintf(line, sizeof line, "%d %d %.6f %.0f %.4f\n", p, node, dt_s, (double)bytes, cpu);
  if (write(out_fd, line, (size_t)n) != n) return 2;
  close(fd);
  return 0;
}

int main(int argc, char **argv) {
  for (int a = 1; a < argc; a++) {
    if (!strcmp(argv[a], "--pipelines") && a + 1 < argc) P = atoi(argv[++a]);
    else if (!strcmp(argv[a], "--threads") && a + 1 < argc) T = atoi(argv[++a]);
    else if (!strcmp(argv[a], "--segment-mb") && a + 1 < argc) SEG = (size_t)atol(argv[++a]) << 20;
    else if (!strcmp(argv[a], "--batch-mb") && a + 1 < argc) BATCH = (size_t)atol(argv[++a]) << 20;
    else if (!strcmp(argv[a], "--seconds") && a + 1 < argc) SECONDS = atof(argv[++a]);
    else if (!strcmp(argv[a], "--dma")) DMA = 1;
    else if (!strcmp(argv[a], "--dir") && a + 1 < argc) DIR_ = argv[++a];
    else {
      fprintf(stderr, "usage: %s [--pipelines P] [--threads T] [--segment-mb M] [--batch-mb B] [--seconds S] [--dma] [--dir D]\n", argv[0]);
      return 1;
    }
  }
  if (P < 1 || P > 64 || T < 1 || T > 64) return 1;
  int pfd[2];
  if (pipe(pfd)) return 1;
  pid_t kids[64];
  for (int p = 0; p < P; p++) {
    kids[p] = fork();
    if (kids[p] == 0) {
      close(pfd[0]);
      _exit(pipeline(p, pfd[1]));
    }
  }
  close(pfd[1]);
  int bad = 0;
  for (int p = 0; p < P; p++) {
    int st = 0;
    waitpid(kids[p], &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st)) bad = 1;
  }
  char buf[65536];
  ssize_t n = read(pfd[0], buf, sizeof buf - 1);
  buf[n > 0 ? n : 0] = 0;
  double gbs = 0, cpu = 0, secs = 0, bytes = 0;
  printf("{\"pipelines\": %d, \"threads_per_pipeline\": %d, \"segment_bytes\": %zu, \"batch_bytes\": %zu, "
         "\"dma_stand_in\": %s, \"per_pipeline\": [", P, T, SEG, BATCH, DMA ? "true" : "false");
  int first = 1;
  for (char *s = buf; *s;) {
    int p, node;
    double dt, by, c;
    int used = 0;
    if (sscanf(s, "%d %d %lf %lf %lf\n%n", &p, &node, &dt, &by, &c, &used) != 5 || !used) break;
    s += used;
    printf("%s{\"pipeline\": %d, \"node\": %d, \"GBps\": %.2f, \"cpu_s_per_GB\": %.4f}", first ? "" : ", ", p, node,
           by / dt / 1e9, c / (by / 1e9));
    first = 0;
    gbs += by / dt / 1e9;
    cpu += c;
    bytes += by;
    secs = dt > secs ? dt : secs;
  }
  long q = -1, per = 100000;
  FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r");
  if (f) {
    char qs[32];
    if (fscanf(f, "%31s %ld", qs, &per) == 2 && strcmp(qs, "max")) q = atol(qs);
    fclose(f);
  }
  printf("], \"aggregate_GBps\": %.2f, \"implied_4k_fps\": %.0f, \"cpu_s_per_GB\": %.4f, "
         "\"cpu_quota_cores\": %.2f, \"numa_nodes\": %d, \"ok\": %s}\n", gbs, gbs * 1e9 / 12441600.0,
         bytes > 0 ? cpu / (bytes / 1e9) : 0.0, q > 0 ? (double)q / per : -1.0, nnodes(), bad ? "false" : "true");
  return bad;
}
