// mjg_client: the per-segment `gpu:N` worker process the dispatcher starts for each segment
// (ffmpeg_distributed.py:131-141: segment on stdin, encoded segment on stdout, ffmpeg-style
// progress on stderr, exit code 0 on success), as a thin client of a resident per-GPU encoder
// process (ffmpeg_distributed_amd/resident.py).
//
// A fresh Python worker per segment pays interpreter start, imports, HIP init, the encoder
// context and page-locked buffers (~0.5 s per segment).  This client instead hands
// its three standard descriptors to the resident encoder of its GPU over a Unix socket
// (SCM_RIGHTS), waits for the segment's exit code and exits with it.  The resident process
// reads the segment from the client's stdin, writes the Matroska output to its stdout and the
// progress lines to its stderr, exactly as the per-process worker does, and closes its copies
// of the three descriptors before it answers, so when this process exits the dispatcher sees
// the same end of stream and exit code as from ffmpeg.
//
// If no resident encoder listens (first segment, or it exited after its idle timeout), the
// client starts one, with no descriptor of the segment inherited, and then connects.  This process never touches the GPU, so starting the encoder with fork + exec is
// safe.  The socket lives in the abstract namespace; its name carries the user id, the device,
// the visible-device environment, the process-level MJG_* settings the encoder reads once
// (MJG_LIBRARY, MJG_NUMA_BIND, MJG_SERVE_BATCH_BYTES), and the inode and mtime of the library
// it loads (MJG_LIBRARY or libmjgpu.so beside this client), so a rebuilt library, another
// library or another device mapping gets a new encoder.  The abstract namespace has no file
// permissions, so both sides check the peer: the encoder serves only its uid, and this client
// hands its descriptors only to an encoder of its own uid (SO_PEERCRED).  The encoder's log is
// /tmp/mjg-<uid>/<socket name>.log in a 0700 directory of this user (no symlinks followed).
//
//   mjg_client --device N [--python PATH] [--idle SECONDS] [--] <remote_args...>
//   mjg_client --device N --shutdown        (asks a running encoder to exit; 0 if none runs)
//   mjg_client --device N --socket-name     (prints the encoder's socket name)
//
// Wire format (little-endian), client -> encoder, one message with SCM_RIGHTS {0, 1, 2}:
//   "MJG2" u32 total_bytes u32 kind (0 encode, 1 shutdown) u32 nargs u32 nenv, then nargs
//   NUL-terminated arguments and nenv NUL-terminated "NAME=VALUE" strings (the MJG_* settings
//   of this process's environment); encoder -> client: the byte 'A' once the request is read
//   (before any of the segment is), then the i32 exit code.  A connection that ends before the
//   'A' (an encoder closing its socket at its idle timeout while this client queued) touched
//   nothing of the segment: the client connects again, starting an encoder if none listens.
//   Any other first byte is a hard error (never a retry: the request may have been consumed).
//   "MJG2" (r05): the 'A' acknowledgement; an encoder of the older "MJG1" protocol refuses the
//   request as malformed and closes the connection before any byte, which the retry loop then
//   meets three times and reports.
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <sys/un.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

extern char **environ;

static const char *kMagic = "MJG2";

static int die(const char *dev, const char *msg, int err) {
  if (err)
    fprintf(stderr, "gpu:%s: %s: %s\n", dev, msg, strerror(err));
  else
    fprintf(stderr, "gpu:%s: %s\n", dev, msg);
  return 1;
}

// FNV-1a over a string (visible-device environment in the socket name)
static uint64_t fnv(uint64_t h, const char *s) {
  for (; s && *s; s++) h = (h ^ (unsigned char)*s) * 1099511628211ull;
  return h ^ 0xffu;
}

// directory of this executable (the package directory: libmjgpu.so sits beside it)
static int self_dir(char *out, size_t cap) {
  ssize_t n = readlink("/proc/self/exe", out, cap - 1);
  if (n <= 0) return -1;
  out[n] = 0;
  char *s = strrchr(out, '/');
  if (!s) return -1;
  *s = 0;
  return 0;
}

static int sock_name(const char *dev, const char *pkg, char *name, size_t cap) {
  char lib[4200];
  const char *ml = getenv("MJG_LIBRARY");  // _lib.py loads this one instead when set
  if (ml && *ml)
    snprintf(lib, sizeof lib, "%s", ml);
  else
    snprintf(lib, sizeof lib, "%s/libmjgpu.so", pkg);
  struct stat st;
  if (stat(lib, &st) != 0) return -1;
  uint64_t h = 1469598103934665603ull;
  h = fnv(h, getenv("HIP_VISIBLE_DEVICES"));
  h = fnv(h, getenv("ROCR_VISIBLE_DEVICES"));
  h = fnv(h, getenv("CUDA_VISIBLE_DEVICES"));
  h = fnv(h, getenv("GPU_DEVICE_ORDINAL"));
  // settings the encoder process reads once at import (worker.py, _lib.py)
  h = fnv(h, ml);
  h = fnv(h, getenv("MJG_NUMA_BIND"));
  h = fnv(h, getenv("MJG_SERVE_BATCH_BYTES"));
  // read by the library at mjg_open, in the encoder's process
  h = fnv(h, getenv("MJG_MERGE"));
  h = fnv(h, getenv("MJG_MERGE_HOLD"));
  h = fnv(h, getenv("MJG_TIMING_NOTAIL"));
  h = fnv(h, kMagic);  // the protocol: a client never meets an encoder of another wire format
  snprintf(name, cap, "mjg-gpu-%u-%s-%llx-%llx-%llx", (unsigned)getuid(), dev, (unsigned long long)st.st_ino,
           (unsigned long long)st.st_mtim.tv_sec * 1000000000ull + (unsigned long long)st.st_mtim.tv_nsec,
           (unsigned long long)h);
  return 0;
}

static int try_connect(const char *name) {
  int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -errno;
  struct sockaddr_un a;
  memset(&a, 0, sizeof a);
  a.sun_family = AF_UNIX;
  const size_t n = strlen(name);
  memcpy(a.sun_path + 1, name, n);  // abstract namespace: leading NUL
  if (connect(fd, (struct sockaddr *)&a, (socklen_t)(offsetof(struct sockaddr_un, sun_path) + 1 + n)) != 0) {
    const int e = errno;
    close(fd);
    return -e;
  }
  // the abstract namespace has no permissions: hand descriptors only to our own uid
  struct ucred cr;
  socklen_t cl = sizeof cr;
  if (getsockopt(fd, SOL_SOCKET, SO_PEERCRED, &cr, &cl) != 0 || cr.uid != getuid()) {
    close(fd);
    return -EACCES;
  }
  return fd;
}

// /tmp/mjg-<uid>: created 0700, and used only when it is a real directory of this user with no
// access for others (not a symlink another user planted)
static int log_dir(char *out, size_t cap) {
  snprintf(out, cap, "/tmp/mjg-%u", (unsigned)getuid());
  if (mkdir(out, 0700) != 0 && errno != EEXIST) return -1;
  struct stat st;
  if (lstat(out, &st) != 0 || !S_ISDIR(st.st_mode) || st.st_uid != getuid() || (st.st_mode & 077)) return -1;
  return 0;
}

// Start the resident encoder: cwd = the package's parent (python -m finds the package there),
// stdin /dev/null, stdout/stderr to its log (never the segment's pipes: the dispatcher waits for
// EOF on this process's stderr), no other descriptor inherited.  It stays in the caller's
// process group (no setsid): whoever stops the dispatcher's job by its group stops the encoder
// too, and otherwise it ends after its idle timeout.
static pid_t spawn(const char *python, const char *pkg, const char *dev, const char *name, const char *idle,
                   const char *logp) {
  char root[4096];
  snprintf(root, sizeof root, "%s", pkg);
  char *s = strrchr(root, '/');
  if (!s) return -1;
  *s = 0;
  const pid_t pid = fork();
  if (pid != 0) return pid;
  const int nul = open("/dev/null", O_RDONLY);
  int log = *logp ? open(logp, O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC | O_NOFOLLOW, 0600) : -1;
  struct stat st;
  if (log >= 0 && (fstat(log, &st) != 0 || !S_ISREG(st.st_mode) || st.st_uid != getuid())) {
    close(log);
    log = -1;
  }
  if (log < 0) log = open("/dev/null", O_WRONLY);
  if (nul < 0 || chdir(root) != 0) _exit(126);
  dup2(nul, 0);
  dup2(log, 1);
  dup2(log, 2);
  for (int fd = 3; fd < 1024; fd++) close(fd);
  const char *argv[] = {python, "-m", "ffmpeg_distributed_amd.resident", "--device", dev, "--socket", name,
                        "--idle", idle, NULL};
  execvp(python, (char *const *)argv);
  _exit(127);
}

static int send_all_fds(int sk, const char *buf, size_t len, int with_fds) {
  size_t off = 0;
  while (off < len) {
    struct iovec iov = {(void *)(buf + off), len - off};
    struct msghdr m;
    memset(&m, 0, sizeof m);
    m.msg_iov = &iov;
    m.msg_iovlen = 1;
    union {
      char b[CMSG_SPACE(3 * sizeof(int))];
      struct cmsghdr align;
    } u;
    if (with_fds && off == 0) {
      memset(&u, 0, sizeof u);
      m.msg_control = u.b;
      m.msg_controllen = sizeof u.b;
      struct cmsghdr *c = CMSG_FIRSTHDR(&m);
      c->cmsg_level = SOL_SOCKET;
      c->cmsg_type = SCM_RIGHTS;
      c->cmsg_len = CMSG_LEN(3 * sizeof(int));
      const int fds[3] = {0, 1, 2};
      memcpy(CMSG_DATA(c), fds, sizeof fds);
    }
    const ssize_t k = sendmsg(sk, &m, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    off += (size_t)k;
  }
  return 0;
}

static void put_u32(char *p, uint32_t v) {
  p[0] = (char)v;
  p[1] = (char)(v >> 8);
  p[2] = (char)(v >> 16);
  p[3] = (char)(v >> 24);
}

int main(int argc, char **argv) {
  const char *dev = NULL, *python = "python3", *idle = "30";
  int shutdown_req = 0, print_name = 0, a = 1;
  for (; a < argc; a++) {
    if (!strcmp(argv[a], "--device") && a + 1 < argc)
      dev = argv[++a];
    else if (!strcmp(argv[a], "--python") && a + 1 < argc)
      python = argv[++a];
    else if (!strcmp(argv[a], "--idle") && a + 1 < argc)
      idle = argv[++a];
    else if (!strcmp(argv[a], "--shutdown"))
      shutdown_req = 1;
    else if (!strcmp(argv[a], "--socket-name"))
      print_name = 1;
    else if (!strcmp(argv[a], "--")) {
      a++;
      break;
    } else
      break;  // the first remote argument
  }
  if (!dev || !*dev || strspn(dev, "0123456789") != strlen(dev)) return die("?", "usage: mjg_client --device N [--] ARGS", 0);
  signal(SIGPIPE, SIG_IGN);
  char pkg[4096], name[200];
  if (self_dir(pkg, sizeof pkg) != 0) return die(dev, "cannot resolve /proc/self/exe", errno);
  if (sock_name(dev, pkg, name, sizeof name) != 0) return die(dev, "libmjgpu.so not found beside mjg_client", errno);
  if (print_name) {
    printf("%s\n", name);
    return 0;
  }

  char logp[4400] = "", ldir[64];
  if (log_dir(ldir, sizeof ldir) == 0) snprintf(logp, sizeof logp, "%s/%s.log", ldir, name);

  // with MJG_WORKER_TRACE=1 the start time goes along (MJG_CLIENT_T0, CLOCK_MONOTONIC ns): the
  // encoder's trace line then splits process start + hand-off from the encode (worker.py)
  {
    const char *t = getenv("MJG_WORKER_TRACE");
    if (t && !strcmp(t, "1")) {
      struct timespec ts;
      clock_gettime(CLOCK_MONOTONIC, &ts);
      char v[32];
      snprintf(v, sizeof v, "%lld", (long long)ts.tv_sec * 1000000000ll + ts.tv_nsec);
      setenv("MJG_CLIENT_T0", v, 1);
    }
  }
  // request: header, arguments, MJG_* environment
  size_t len = 20, nargs = (size_t)(argc - a), nenv = 0;
  for (int i = a; i < argc; i++) len += strlen(argv[i]) + 1;
  for (char **e = environ; *e; e++)
    if (!strncmp(*e, "MJG_", 4)) {
      len += strlen(*e) + 1;
      nenv++;
    }
  char *buf = malloc(len);
  if (!buf) return die(dev, "out of memory", 0);
  memcpy(buf, kMagic, 4);
  put_u32(buf + 4, (uint32_t)len);
  put_u32(buf + 8, shutdown_req ? 1u : 0u);
  put_u32(buf + 12, (uint32_t)nargs);
  put_u32(buf + 16, (uint32_t)nenv);
  char *p = buf + 20;
  for (int i = a; i < argc; i++) {
    const size_t n = strlen(argv[i]) + 1;
    memcpy(p, argv[i], n);
    p += n;
  }
  for (char **e = environ; *e; e++)
    if (!strncmp(*e, "MJG_", 4)) {
      const size_t n = strlen(*e) + 1;
      memcpy(p, *e, n);
      p += n;
    }

  int sk = -1;
  pid_t child = -1;
  for (int attempt = 0;; attempt++) {
    sk = try_connect(name);
    if (sk == -EACCES) return die(dev, "the encoder socket belongs to another user; not sending the segment", 0);
    if (sk < 0 && shutdown_req) return 0;  // nothing runs
    if (sk < 0) {
      child = spawn(python, pkg, dev, name, idle, logp);
      if (child < 0) return die(dev, "cannot start the resident encoder", errno);
      const struct timespec ts = {0, 2000000};  // 2 ms
      for (int i = 0; i < 60000 && sk < 0; i++) {  // up to ~2 min (first start: imports + HIP init)
        nanosleep(&ts, NULL);
        sk = try_connect(name);
        if (sk == -EACCES) return die(dev, "the encoder socket belongs to another user; not sending the segment", 0);
        int st;
        if (sk < 0 && child > 0 && waitpid(child, &st, WNOHANG) == child) {
          child = -1;  // exited: lost the bind race to another encoder (exit 0), or failed
          if (!(WIFEXITED(st) && WEXITSTATUS(st) == 0)) {
            fprintf(stderr, "gpu:%s: resident encoder failed to start (log: %s)\n", dev, *logp ? logp : "none");
            return 1;
          }
        }
      }
      if (sk < 0) return die(dev, "resident encoder did not come up", -sk);
    }
    const int rc_send = send_all_fds(sk, buf, len, !shutdown_req);
    unsigned char ack = 0;
    ssize_t k = -1;
    int rerr = 0;
    if (rc_send == 0) {
      do k = read(sk, &ack, 1);
      while (k < 0 && errno == EINTR);
      rerr = k < 0 ? errno : 0;
    }
    if (k == 1 && ack == 'A') break;
    close(sk);
    if (k == 1)  // a byte that is not the acknowledgement: another protocol; never resend
      return die(dev, "the resident encoder answered outside the MJG2 protocol", 0);
    if (k < 0 && rerr != ECONNRESET && rerr != EPIPE)
      return die(dev, "reading the resident encoder's acknowledgement", rerr);
    // EOF / reset before the 'A': the encoder closed this connection unread (idle exit);
    // nothing of the segment was consumed, so connect again (a few times at most)
    if (attempt == 3) return die(dev, "the resident encoder keeps closing the connection", rc_send < 0 ? -rc_send : 0);
    const struct timespec ts = {0, 20000000};  // 20 ms
    nanosleep(&ts, NULL);
  }
  free(buf);

  unsigned char r[4];
  size_t got = 0;
  while (got < 4) {
    const ssize_t k = read(sk, r + got, 4 - got);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return die(dev, "resident encoder exited during the segment", k < 0 ? errno : 0);
    got += (size_t)k;
  }
  close(sk);
  if (child > 0) waitpid(child, NULL, WNOHANG);
  const int32_t rc = (int32_t)((uint32_t)r[0] | ((uint32_t)r[1] << 8) | ((uint32_t)r[2] << 16) | ((uint32_t)r[3] << 24));
  return rc < 0 || rc > 255 ? 1 : rc;
}
