// Standalone sanitizer test of the host runtime (race detection / sanitizers).
//
// Built with -fsanitize=address,undefined (tests/test_native_sanitizers.py) and run as
// p forked processes sharing one anonymous MAP_SHARED mapping, exactly the layout the
// /dev/shm engine uses.  Checks every collective of csrc/host/host_ops.cpp against a scalar
// reference, including pieces larger than a slot (multi-round paths) and ragged blocks.
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "mp4x/ops.h"

extern "C" {
int mp4x_host_reduce(int dtype, int op, void* out, const void* const* ins, int nin, int64_t n, int nthreads);
void* mp4x_shm_attach(void* base, int rank, int p, int64_t slot_bytes, int nthreads, double timeout_s);
void mp4x_shm_detach(void* h);
int mp4x_shm_allreduce(void* h, int dtype, int op, void* buf, int64_t n);
int mp4x_shm_reduce_scatter(void* h, int dtype, int op, void* buf, const int64_t* froms, const int64_t* tos);
int mp4x_shm_allgather(void* h, int es, void* buf, const int64_t* froms, const int64_t* tos);
int mp4x_shm_broadcast(void* h, int es, void* buf, int64_t frm, int64_t to, int root);
}

static double val(int rank, int64_t i) { return (double)((rank * 7 + i * 3) % 11) - 5.0; }

#define CHECK(c, ...)                                  \
  do {                                                 \
    if (!(c)) {                                        \
      fprintf(stderr, "FAIL rank %d: ", rank);         \
      fprintf(stderr, __VA_ARGS__);                    \
      fprintf(stderr, "\n");                           \
      _exit(1);                                        \
    }                                                  \
  } while (0)

static void run_rank(void* base, int rank, int p, int64_t slot, int64_t n) {
  void* h = mp4x_shm_attach(base, rank, p, slot, 3, 60.0);
  // allreduce SUM (n larger than one slot -> several rounds)
  std::vector<double> a(n);
  for (int64_t i = 0; i < n; ++i) a[i] = val(rank, i);
  CHECK(mp4x_shm_allreduce(h, MP4X_F64, MP4X_SUM, a.data(), n) == 0, "allreduce rc");
  for (int64_t i = 0; i < n; ++i) {
    double e = 0;
    for (int r = 0; r < p; ++r) e += val(r, i);
    CHECK(a[i] == e, "allreduce[%ld] %f != %f", (long)i, a[i], e);
  }
  // ragged reduce-scatter (int32 MAX) and allgather
  std::vector<int64_t> f(p), t(p);
  int64_t off = 0;
  for (int r = 0; r < p; ++r) {
    f[r] = off;
    off += (n / p) + (r % 3) * 17 - (r == 0 ? 0 : 5);
    if (off > n) off = n;
    t[r] = off;
  }
  std::vector<int32_t> b(n);
  for (int64_t i = 0; i < n; ++i) b[i] = (int32_t)(val(rank, i) * 3);
  CHECK(mp4x_shm_reduce_scatter(h, MP4X_I32, MP4X_MAX, b.data(), f.data(), t.data()) == 0, "rs rc");
  for (int64_t i = f[rank]; i < t[rank]; ++i) {
    int32_t e = INT32_MIN;
    for (int r = 0; r < p; ++r) e = std::max(e, (int32_t)(val(r, i) * 3));
    CHECK(b[i] == e, "rs[%ld]", (long)i);
  }
  std::vector<int16_t> c(n, -1);
  for (int64_t i = f[rank]; i < t[rank]; ++i) c[i] = (int16_t)rank;
  CHECK(mp4x_shm_allgather(h, 2, c.data(), f.data(), t.data()) == 0, "ag rc");
  for (int r = 0; r < p; ++r)
    for (int64_t i = f[r]; i < t[r]; ++i) CHECK(c[i] == r, "ag[%ld]", (long)i);
  // broadcast from the last rank
  std::vector<int8_t> d(n, (int8_t)(rank == p - 1 ? 7 : 0));
  CHECK(mp4x_shm_broadcast(h, 1, d.data(), 3, n - 2, p - 1) == 0, "bc rc");
  for (int64_t i = 3; i < n - 2; ++i) CHECK(d[i] == 7, "bc[%ld]", (long)i);
  mp4x_shm_detach(h);
}

// sum of two int64 inputs over n elements through mp4x_host_reduce with nt threads, `reps` times
static void pool_check(int64_t n, int nt, int reps) {
  const int rank = -1;                               // (CHECK's report)
  std::vector<int64_t> x(n), y(n), z(n);
  for (int64_t i = 0; i < n; ++i) {
    x[i] = i;
    y[i] = 3 * i + 1;
  }
  const void* ins[2] = {x.data(), y.data()};
  for (int r = 0; r < reps; ++r) {
    const int w = 1 + (nt + r) % (nt + 2);           // widths 1..nt+2
    CHECK(mp4x_host_reduce(MP4X_I64, MP4X_SUM, z.data(), ins, 2, n, w) == 0, "pool reduce");
    for (int64_t i = 0; i < n; i += 997) CHECK(z[i] == 4 * i + 1, "pool reduce value at %lld", (long long)i);
    CHECK(z[n - 1] == 4 * (n - 1) + 1, "pool reduce tail");
  }
}

int main(int argc, char** argv) {
  const int p = argc > 1 ? atoi(argv[1]) : 4;
  const int64_t n = argc > 2 ? atoll(argv[2]) : 100003;
  const int64_t slot = 1 << 16;   // small slots: forces multi-round pieces
  // local reduce kernel, every op on int64 incl. *_LOC
  {
    int rank = -1;
    std::vector<int64_t> x(1000), y(1000), z(1000);
    for (int i = 0; i < 1000; ++i) {
      x[i] = ((int64_t)(i % 7) << 32) | 1;
      y[i] = ((int64_t)(i % 5) << 32) | 2;
    }
    const void* ins[2] = {x.data(), y.data()};
    for (int op : {MP4X_SUM, MP4X_MAX, MP4X_MIN, MP4X_PROD, MP4X_BAND, MP4X_BOR, MP4X_BXOR, MP4X_IMAXLOC,
                   MP4X_IMINLOC})
      CHECK(mp4x_host_reduce(MP4X_I64, op, z.data(), ins, 2, 1000, 4) == 0, "reduce op %d", op);
    CHECK(mp4x_host_reduce(MP4X_F32, MP4X_BXOR, z.data(), ins, 2, 10, 1) == MP4X_E_UNSUPPORTED, "float xor");
  }
  // the persistent fan-out pool: many jobs back to back, varying widths, two concurrent callers
  // (one gets the pool, the other the spawn fallback); the forked ranks below then get a fresh
  // pool of their own (the parent's workers do not exist in a child)
  pool_check(1 << 20, 4, 50);
  {
    std::thread a([] { pool_check((1 << 20) + 7, 5, 40); });
    pool_check((1 << 19) + 3, 3, 40);
    a.join();
  }
  size_t bytes = 4096 + (size_t)p * slot;
  void* base = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (base == MAP_FAILED) return 2;
  memset(base, 0, bytes);
  std::vector<pid_t> kids;
  for (int r = 0; r < p; ++r) {
    pid_t pid = fork();
    if (pid == 0) {
      pool_check(1 << 18, 3, 5);                   // pool after fork: a fresh one in the child
      run_rank(base, r, p, slot, n);
      _exit(0);
    }
    kids.push_back(pid);
  }
  int bad = 0;
  for (pid_t k : kids) {
    int st = 0;
    waitpid(k, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) bad++;
  }
  munmap(base, bytes);
  printf(bad ? "FAILED %d ranks\n" : "OK p=%d\n", bad ? bad : p);
  return bad ? 1 : 0;
}
