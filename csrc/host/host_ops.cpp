// mp4x host runtime (C++17, std::thread): CPU reduction kernels + the shared-memory intra-node
// data plane.
//
// Reference hot loops replaced here:
//   * the per-element reduce-on-receive / thread reduce loops
//     (/root/reference/src/main/java/com/fenbi/mp4j/operand/DoubleOperand.java:196, :453)
//     -> mp4x_host_reduce: multi-input, multi-threaded, auto-vectorised (AVX2) loops;
//   * the per-message TCP transport for ranks that share a host
//     (ProcessCommSlave.java:89-127, 391-425) -> a /dev/shm segment with one slot per rank
//     and a process-shared sense-counting barrier.  Collectives become memcpy/reduce passes
//     at memory bandwidth:
//        allreduce      = copy-in, barrier, rank r reduces chunk r over all slots (rank order),
//                         barrier, copy every chunk out, barrier  (the CPU twin of the IPC
//                         two-shot kernel in csrc/runtime/ipc.hip)
//        reduce-scatter = the first half, ragged blocks;  allgather = slot copy-out;
//        broadcast      = root copy-in + copy-out.
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <type_traits>
#include <vector>

#include <cerrno>
#include <climits>
#include <csignal>
#include <cstdio>
#include <cstdlib>

#include <linux/futex.h>
#include <sched.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include "mp4x/ops.h"

namespace {

long futex_word(std::atomic<uint32_t>* addr, int op, uint32_t val) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), op | FUTEX_PRIVATE_FLAG, val, nullptr, nullptr, 0);
}

// Persistent fan-out pool (no OpenMP: no runtime state must survive a fork in the rank launchers,
// and torch ships its own libgomp).  A job splits [0, nb) over nt threads, the caller runs chunk
// 0; the workers wait on a generation word (short spin, then a futex), so a job costs one wake,
// not nt-1 thread creations (the shm engine runs 4 fan-outs per 16 MiB piece: spawning was ~1/3
// of an 800 MB allreduce on the box).  Every worker acknowledges every job (those past nt just
// count), so the caller's wait covers them all and no late count leaks into the next job; workers
// are only added under the job lock, between jobs.  One job at a time: a concurrent caller, or a
// forked child (whose copy of the pool has no threads), falls back to spawning.
struct Pool {
  std::mutex job;
  std::atomic<uint32_t> gen{0};
  std::atomic<uint32_t> done{0};
  std::atomic<uint32_t> sleepers{0};
  int nworkers = 0;                         // detached worker threads 1..nworkers (job lock)
  int nt = 0;                               // threads in the current job (incl. the caller)
  int64_t nb = 0;
  void (*fn)(void*, int64_t) = nullptr;
  void* ctx = nullptr;
  pid_t pid = 0;

  void run_range(int t) const {
    const int64_t lo = nb * t / nt, hi = nb * (t + 1) / nt;
    for (int64_t b = lo; b < hi; ++b) fn(ctx, b);
  }

  void worker(int t, uint32_t seen) {
    for (;;) {
      for (int i = 0; gen.load(std::memory_order_acquire) == seen; ++i) {
        if (i < 4096) {
          __builtin_ia32_pause();
          continue;
        }
        sleepers.fetch_add(1, std::memory_order_seq_cst);
        if (gen.load(std::memory_order_seq_cst) == seen) futex_word(&gen, FUTEX_WAIT, seen);
        sleepers.fetch_sub(1, std::memory_order_seq_cst);
      }
      ++seen;                               // exactly one job per generation (the caller waits)
      if (t < nt) run_range(t);
      done.fetch_add(1, std::memory_order_acq_rel);
    }
  }
};

Pool* g_pool = nullptr;
std::mutex g_pool_mu;

Pool* the_pool() {
  std::lock_guard<std::mutex> g(g_pool_mu);
  if (!g_pool || g_pool->pid != getpid()) {   // first use, or a forked child: a fresh pool (leak the old)
    g_pool = new Pool();
    g_pool->pid = getpid();
  }
  return g_pool;
}

template <typename F>
void parallel_for(int64_t nb, int nt, F&& body) {
  if (nt <= 1 || nb <= 1) {
    for (int64_t b = 0; b < nb; ++b) body(b);
    return;
  }
  if (nt > nb) nt = (int)nb;
  Pool* p = the_pool();
  std::unique_lock<std::mutex> job(p->job, std::try_to_lock);
  if (!job.owns_lock()) {                      // pool busy: spawn for this job
    std::vector<std::thread> th;
    th.reserve(nt - 1);
    auto run = [&](int t) {
      const int64_t lo = nb * t / nt, hi = nb * (t + 1) / nt;
      for (int64_t b = lo; b < hi; ++b) body(b);
    };
    for (int t = 1; t < nt; ++t) th.emplace_back(run, t);
    run(0);
    for (auto& x : th) x.join();
    return;
  }
  const uint32_t g = p->gen.load(std::memory_order_relaxed);
  while (p->nworkers < nt - 1) {               // grow between jobs: new workers wait for g + 1
    const int t = ++p->nworkers;
    std::thread([p, t, g] { p->worker(t, g); }).detach();
  }
  using B = typename std::remove_reference<F>::type;
  p->fn = [](void* c, int64_t b) { (*static_cast<B*>(c))(b); };
  p->ctx = const_cast<void*>(static_cast<const void*>(&body));
  p->nb = nb;
  p->nt = nt;
  p->done.store(0, std::memory_order_relaxed);
  p->gen.store(g + 1, std::memory_order_seq_cst);
  if (p->sleepers.load(std::memory_order_seq_cst)) futex_word(&p->gen, FUTEX_WAKE, INT_MAX);
  p->run_range(0);
  const uint32_t all = (uint32_t)p->nworkers;
  for (int i = 0; p->done.load(std::memory_order_acquire) != all; ++i) {
    if (i < 65536) __builtin_ia32_pause();
    else sched_yield();                        // a worker descheduled by the cpu quota
  }
}

template <typename T> struct Uns { using U = T; };
template <> struct Uns<int64_t> { using U = uint64_t; };
template <> struct Uns<int32_t> { using U = uint32_t; };
template <> struct Uns<int16_t> { using U = uint16_t; };
template <> struct Uns<int8_t> { using U = uint8_t; };

template <typename T, int OP>
inline T comb(T a, T b) {
  if constexpr (OP == MP4X_SUM) {
    if constexpr (std::is_floating_point<T>::value) return a + b;
    else { using U = typename Uns<T>::U; return (T)((U)a + (U)b); }
  } else if constexpr (OP == MP4X_PROD) {
    if constexpr (std::is_floating_point<T>::value) return a * b;
    else { using U = typename Uns<T>::U; return (T)((U)a * (U)b); }
  } else if constexpr (OP == MP4X_MAX) {
    if constexpr (std::is_floating_point<T>::value) return (a != a) ? a : ((b != b) ? b : (a >= b ? a : b));
    else return a >= b ? a : b;
  } else if constexpr (OP == MP4X_MIN) {
    if constexpr (std::is_floating_point<T>::value) return (a != a) ? a : ((b != b) ? b : (a <= b ? a : b));
    else return a <= b ? a : b;
  } else if constexpr (OP == MP4X_BAND) {
    return a & b;
  } else if constexpr (OP == MP4X_BOR) {
    return a | b;
  } else if constexpr (OP == MP4X_BXOR) {
    return a ^ b;
  } else if constexpr (OP == MP4X_FMAXLOC || OP == MP4X_FMINLOC) {
    uint64_t ua, ub;
    std::memcpy(&ua, &a, 8);
    std::memcpy(&ub, &b, 8);
    uint32_t ha = (uint32_t)(ua >> 32), hb = (uint32_t)(ub >> 32);
    float va, vb;
    std::memcpy(&va, &ha, 4);
    std::memcpy(&vb, &hb, 4);
    bool keep = OP == MP4X_FMAXLOC ? (va >= vb) : (va <= vb);
    return keep ? a : b;
  } else {
    int32_t va = (int32_t)((uint64_t)a >> 32), vb = (int32_t)((uint64_t)b >> 32);
    bool keep = OP == MP4X_IMAXLOC ? (va >= vb) : (va <= vb);
    return keep ? a : b;
  }
}

template <typename T, int OP>
constexpr bool valid() {
  if (OP <= MP4X_PROD) return true;
  if (OP <= MP4X_BXOR) return !std::is_floating_point<T>::value;
  if (OP == MP4X_FMAXLOC || OP == MP4X_FMINLOC) return std::is_same<T, double>::value;
  return std::is_same<T, int64_t>::value;
}

// out[i] = op(in[0][i], ..., in[k-1][i]) on [lo, hi); out may alias in[0].
template <typename T, int OP>
void reduce_range(T* out, const T* const* ins, int nin, int64_t lo, int64_t hi) {
  const T* a = ins[0];
  if (nin == 1) {
    if (out != a) std::memcpy(out + lo, a + lo, (hi - lo) * sizeof(T));
    return;
  }
  const T* b = ins[1];
  for (int64_t i = lo; i < hi; ++i) out[i] = comb<T, OP>(a[i], b[i]);
  for (int k = 2; k < nin; ++k) {
    const T* c = ins[k];
    for (int64_t i = lo; i < hi; ++i) out[i] = comb<T, OP>(out[i], c[i]);
  }
}

template <typename T, int OP>
int reduce_par(void* out, const void* const* ins, int nin, int64_t n, int nthreads) {
  if constexpr (!valid<T, OP>()) {
    return MP4X_E_UNSUPPORTED;
  } else {
    const T* const* in = reinterpret_cast<const T* const*>(ins);
    T* o = reinterpret_cast<T*>(out);
    // split into cache-sized blocks so the k-input passes stay in L2
    const int64_t blk = 1 << 15;
    const int64_t nb = (n + blk - 1) / blk;
    if (nthreads <= 1 || n < (1 << 16)) {
      for (int64_t b = 0; b < nb; ++b) reduce_range<T, OP>(o, in, nin, b * blk, std::min(n, (b + 1) * blk));
      return 0;
    }
    parallel_for(nb, nthreads, [&](int64_t b) { reduce_range<T, OP>(o, in, nin, b * blk, std::min(n, (b + 1) * blk)); });
    return 0;
  }
}

template <typename T>
int reduce_dt(int op, void* out, const void* const* ins, int nin, int64_t n, int nt) {
  switch (op) {
    case MP4X_SUM: return reduce_par<T, MP4X_SUM>(out, ins, nin, n, nt);
    case MP4X_MAX: return reduce_par<T, MP4X_MAX>(out, ins, nin, n, nt);
    case MP4X_MIN: return reduce_par<T, MP4X_MIN>(out, ins, nin, n, nt);
    case MP4X_PROD: return reduce_par<T, MP4X_PROD>(out, ins, nin, n, nt);
    case MP4X_BAND: return reduce_par<T, MP4X_BAND>(out, ins, nin, n, nt);
    case MP4X_BOR: return reduce_par<T, MP4X_BOR>(out, ins, nin, n, nt);
    case MP4X_BXOR: return reduce_par<T, MP4X_BXOR>(out, ins, nin, n, nt);
    case MP4X_FMAXLOC: return reduce_par<T, MP4X_FMAXLOC>(out, ins, nin, n, nt);
    case MP4X_FMINLOC: return reduce_par<T, MP4X_FMINLOC>(out, ins, nin, n, nt);
    case MP4X_IMAXLOC: return reduce_par<T, MP4X_IMAXLOC>(out, ins, nin, n, nt);
    case MP4X_IMINLOC: return reduce_par<T, MP4X_IMINLOC>(out, ins, nin, n, nt);
    default: return MP4X_E_BADARG;
  }
}

int esize(int dtype) {
  switch (dtype) {
    case MP4X_F64: case MP4X_I64: return 8;
    case MP4X_F32: case MP4X_I32: return 4;
    case MP4X_I16: case MP4X_BF16: case MP4X_F16: return 2;
    case MP4X_I8: case MP4X_U8: return 1;
    default: return 0;
  }
}

int host_reduce(int dtype, int op, void* out, const void* const* ins, int nin, int64_t n, int nt) {
  if (n <= 0) return 0;
  if (nin < 1 || !out) return MP4X_E_BADARG;
  switch (dtype) {
    case MP4X_F64: return reduce_dt<double>(op, out, ins, nin, n, nt);
    case MP4X_F32: return reduce_dt<float>(op, out, ins, nin, n, nt);
    case MP4X_I64: return reduce_dt<int64_t>(op, out, ins, nin, n, nt);
    case MP4X_I32: return reduce_dt<int32_t>(op, out, ins, nin, n, nt);
    case MP4X_I16: return reduce_dt<int16_t>(op, out, ins, nin, n, nt);
    case MP4X_I8: return reduce_dt<int8_t>(op, out, ins, nin, n, nt);
    case MP4X_U8: return reduce_dt<uint8_t>(op, out, ins, nin, n, nt);
    default: return MP4X_E_UNSUPPORTED;
  }
}

void par_copy(void* dst, const void* src, int64_t bytes, int nt) {
  if (bytes <= 0 || dst == src) return;
  if (nt <= 1 || bytes < (1 << 20)) {
    std::memcpy(dst, src, bytes);
    return;
  }
  const int64_t blk = 1 << 20;
  const int64_t nb = (bytes + blk - 1) / blk;
  parallel_for(nb, nt, [&](int64_t b) {
    int64_t lo = b * blk, hi = std::min(bytes, lo + blk);
    std::memcpy((char*)dst + lo, (const char*)src + lo, hi - lo);
  });
}

// ---------------------------------------------------------------- sense-counting barrier
// Arrive: fetch_add on `count`; the last arriver resets it and bumps `gen`.  Waiters spin a
// few `pause`s (short meetings: ~2 us for 2 threads), yield a little, then sleep on a futex on
// `gen` (long meetings: no core burnt while a peer does real work, e.g. the root thread's
// process-level collective).  `sleepers` lets the releaser skip the wake syscall when nobody
// sleeps; both sides use seq_cst so a wake-up is never lost.  Process-shared for the /dev/shm
// engine (shared futex), process-private for thread teams.
struct BarrierWords {
  std::atomic<uint32_t>* count;
  std::atomic<uint32_t>* gen;
  std::atomic<uint32_t>* abort;
  std::atomic<uint32_t>* sleepers;
  uint32_t n;
  double timeout_s;
  bool shared;
  // optional liveness probe, polled while sleeping (shm engine: did a peer PROCESS exit?)
  bool (*peer_dead)(const void*) = nullptr;
  const void* ctx = nullptr;
};

static inline long futex_op(std::atomic<uint32_t>* addr, int op, uint32_t val, const timespec* ts, bool shared) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), shared ? op : (op | FUTEX_PRIVATE_FLAG), val, ts,
                 nullptr, 0);
}

static void barrier_wake_all(const BarrierWords& w) {
  if (w.sleepers->load(std::memory_order_seq_cst)) futex_op(w.gen, FUTEX_WAKE, INT_MAX, nullptr, w.shared);
}

// 0 released, -1 timed out (aborts the barrier for everyone), -2 aborted, -3 a peer process
// exited (aborts the barrier for everyone).
static int barrier_wait(const BarrierWords& w) {
  if (w.abort->load(std::memory_order_acquire)) return -2;
  const uint32_t g = w.gen->load(std::memory_order_acquire);
  if (w.count->fetch_add(1, std::memory_order_acq_rel) == w.n - 1) {
    w.count->store(0, std::memory_order_relaxed);
    w.gen->fetch_add(1, std::memory_order_seq_cst);
    barrier_wake_all(w);
    return 0;
  }
  auto t0 = std::chrono::steady_clock::now();
  uint64_t spins = 0;
  const timespec nap = {0, 10 * 1000 * 1000};        // re-check abort / timeout every 10 ms
  while (w.gen->load(std::memory_order_acquire) == g) {
    if (w.abort->load(std::memory_order_relaxed)) return -2;
    ++spins;
    if (spins < 64) {                                // keep this spin SHORT (see TBarrier note)
      __builtin_ia32_pause();
      continue;
    }
    if (spins < 96) {
      sched_yield();
      continue;
    }
    w.sleepers->fetch_add(1, std::memory_order_seq_cst);
    if (w.gen->load(std::memory_order_seq_cst) == g) futex_op(w.gen, FUTEX_WAIT, g, &nap, w.shared);
    w.sleepers->fetch_sub(1, std::memory_order_seq_cst);
    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    // every ~100 ms of sleeping: a dead peer never arrives, so fail now instead of at the timeout
    if (w.peer_dead && (spins & 7) == 0 && w.gen->load(std::memory_order_acquire) == g && w.peer_dead(w.ctx)) {
      w.abort->store(1, std::memory_order_release);
      futex_op(w.gen, FUTEX_WAKE, INT_MAX, nullptr, w.shared);
      return -3;
    }
    if (el > w.timeout_s) {
      w.abort->store(1, std::memory_order_release);
      w.gen->fetch_add(0, std::memory_order_seq_cst);
      futex_op(w.gen, FUTEX_WAKE, INT_MAX, nullptr, w.shared);
      return -1;
    }
  }
  return 0;
}

// ---------------------------------------------------------------- shared-memory engine
constexpr int kShmMaxPids = 128;     // ranks beyond this are not liveness-checked

struct alignas(64) ShmHeader {
  std::atomic<uint32_t> count;
  std::atomic<uint32_t> gen;
  std::atomic<uint32_t> abort;
  std::atomic<uint32_t> sleepers;
  uint32_t p;
  int64_t slot_bytes;
  int32_t pid[kShmMaxPids];          // each rank's pid + /proc start time, written at attach
  uint64_t start[kShmMaxPids];
};

// state letter and start time (clock ticks since boot) of `pid` from /proc/<pid>/stat
static bool proc_stat(int pid, char* state, uint64_t* start) {
  char path[64];
  snprintf(path, sizeof(path), "/proc/%d/stat", pid);
  FILE* f = fopen(path, "r");
  if (!f) return false;
  char buf[1024];
  size_t n = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[n] = 0;
  const char* q = strrchr(buf, ')');          // comm may contain spaces: parse after the last ')'
  if (!q) return false;
  // fields after comm: 3 state, 4 ppid, ... 22 starttime
  char st = 0;
  unsigned long long v = 0;
  int field = 2;
  const char* c = q + 1;
  while (*c) {
    while (*c == ' ') ++c;
    if (!*c) break;
    ++field;
    if (field == 3) st = *c;
    if (field == 22) {
      v = strtoull(c, nullptr, 10);
      break;
    }
    while (*c && *c != ' ') ++c;
  }
  if (field != 22) return false;
  *state = st;
  *start = v;
  return true;
}
static_assert(sizeof(ShmHeader) <= 4096, "header");
static_assert(std::atomic<uint32_t>::is_always_lock_free, "process-shared atomics need lock-free");

struct Shm {
  char* base;
  ShmHeader* hdr;
  int rank, p;
  int64_t slot;
  int nt;
  double timeout_s;
  bool watch = false;                // every peer's /proc entry was visible at attach time
  char* slot_ptr(int r) const { return base + 4096 + (int64_t)r * slot; }
};

// A peer whose /proc entry vanished, turned zombie / dead, or now belongs to a different
// process (pid reused: start time differs) will never arrive at the barrier.
static bool shm_peer_dead(const void* ctx) {
  const Shm* s = static_cast<const Shm*>(ctx);
  const int np = s->p < kShmMaxPids ? s->p : kShmMaxPids;
  for (int r = 0; r < np; ++r) {
    if (r == s->rank) continue;
    char st;
    uint64_t t;
    if (!proc_stat(s->hdr->pid[r], &st, &t) || st == 'Z' || st == 'X' || t != s->hdr->start[r]) return true;
  }
  return false;
}

int shm_barrier(Shm* s) {
  ShmHeader* h = s->hdr;
  BarrierWords w{&h->count, &h->gen, &h->abort, &h->sleepers, (uint32_t)s->p, s->timeout_s, true};
  if (s->watch) {
    w.peer_dead = shm_peer_dead;
    w.ctx = s;
  }
  return barrier_wait(w);
}

}  // namespace

extern "C" {

int mp4x_host_reduce(int dtype, int op, void* out, const void* const* ins, int nin, int64_t n, int nthreads) {
  return host_reduce(dtype, op, out, ins, nin, n, nthreads);
}

int mp4x_host_threads(void) { return (int)std::thread::hardware_concurrency(); }

int64_t mp4x_shm_header_bytes(void) { return 4096; }

// rank 0 initialises the header (segment is zero-filled by the creator); everyone attaches.
void* mp4x_shm_attach(void* base, int rank, int p, int64_t slot_bytes, int nthreads, double timeout_s) {
  Shm* s = new Shm;
  s->base = (char*)base;
  s->hdr = reinterpret_cast<ShmHeader*>(base);
  s->rank = rank;
  s->p = p;
  s->slot = slot_bytes;
  s->nt = nthreads > 0 ? nthreads : 1;
  s->timeout_s = timeout_s > 0 ? timeout_s : 300.0;
  if (rank == 0) {
    s->hdr->p = (uint32_t)p;
    s->hdr->slot_bytes = slot_bytes;
  }
  if (rank < kShmMaxPids) {
    char st;
    uint64_t t = 0;
    s->hdr->pid[rank] = (int32_t)getpid();
    s->hdr->start[rank] = proc_stat((int)getpid(), &st, &t) ? t : 0;
  }
  return s;
}

// After every rank attached: turn on peer-death detection in the barrier iff every peer is
// visible in this process's /proc with the start time it published (same pid namespace).
// Returns 1 when enabled, 0 when not (the barrier then relies on its timeout alone).
int mp4x_shm_watch_peers(void* h) {
  Shm* s = (Shm*)h;
  s->watch = false;
  if (s->p > kShmMaxPids) return 0;
  for (int r = 0; r < s->p; ++r) {
    char st;
    uint64_t t;
    if (!proc_stat(s->hdr->pid[r], &st, &t) || t != s->hdr->start[r] || t == 0) return 0;
  }
  s->watch = true;
  return 1;
}

void mp4x_shm_detach(void* h) { delete (Shm*)h; }

int mp4x_shm_barrier(void* h) { return shm_barrier((Shm*)h); }

// In-place allreduce of buf[0, n) (elements) — pieces of one slot each.
int mp4x_shm_allreduce(void* h, int dtype, int op, void* buf, int64_t n) {
  Shm* s = (Shm*)h;
  const int es = esize(dtype);
  if (!es) return MP4X_E_BADARG;
  const int64_t piece = (s->slot / es / s->p) * s->p;   // elements per round, multiple of p
  if (piece <= 0) return MP4X_E_BADARG;
  char* b = (char*)buf;
  std::vector<const void*> ins(s->p);
  for (int64_t off = 0; off < n; off += piece) {
    const int64_t m = std::min(piece, n - off);
    par_copy(s->slot_ptr(s->rank), b + off * es, m * es, s->nt);
    if (int rc = shm_barrier(s)) return rc;
    // my chunk of this piece: the allreduce split (last rank takes the remainder)
    const int64_t avg = m / s->p;
    const int64_t lo = avg * s->rank, hi = s->rank == s->p - 1 ? m : lo + avg;
    if (hi > lo) {
      // reduce in rank order into the caller's buffer (no aliasing with any input slot), then
      // publish the reduced chunk in this rank's slot for the copy-out phase
      for (int j = 0; j < s->p; ++j) ins[j] = s->slot_ptr(j) + lo * es;
      int rc = host_reduce(dtype, op, b + (off + lo) * es, ins.data(), s->p, hi - lo, s->nt);
      if (rc) return rc;
    }
    if (int rc = shm_barrier(s)) return rc;   // every rank finished reading the slots
    if (hi > lo) par_copy(s->slot_ptr(s->rank) + lo * es, b + (off + lo) * es, (hi - lo) * es, s->nt);
    if (int rc = shm_barrier(s)) return rc;
    for (int j = 0; j < s->p; ++j) {
      if (j == s->rank) continue;
      const int64_t jl = avg * j, jh = j == s->p - 1 ? m : jl + avg;
      par_copy(b + (off + jl) * es, s->slot_ptr(j) + jl * es, (jh - jl) * es, s->nt);
    }
    if (int rc = shm_barrier(s)) return rc;
  }
  return 0;
}

// Ragged reduce-scatter: rank r ends with the reduction of every rank's [froms[r], tos[r]).
int mp4x_shm_reduce_scatter(void* h, int dtype, int op, void* buf, const int64_t* froms, const int64_t* tos) {
  Shm* s = (Shm*)h;
  const int es = esize(dtype);
  if (!es) return MP4X_E_BADARG;
  int64_t maxc = 0;
  for (int j = 0; j < s->p; ++j) maxc = std::max(maxc, tos[j] - froms[j]);
  // slot layout per round: p sub-blocks of `q` elements (sub-block j = block j's window)
  const int64_t q = s->slot / es / s->p;
  if (q <= 0) return MP4X_E_BADARG;
  char* b = (char*)buf;
  std::vector<const void*> ins(s->p);
  for (int64_t off = 0; off < maxc; off += q) {
    char* mine = s->slot_ptr(s->rank);
    for (int j = 0; j < s->p; ++j) {
      const int64_t c = tos[j] - froms[j];
      if (off < c) par_copy(mine + j * q * es, b + (froms[j] + off) * es, std::min(q, c - off) * es, s->nt);
    }
    if (int rc = shm_barrier(s)) return rc;
    const int64_t c = tos[s->rank] - froms[s->rank];
    if (off < c) {
      const int64_t m = std::min(q, c - off);
      for (int j = 0; j < s->p; ++j) ins[j] = s->slot_ptr(j) + s->rank * q * es;
      int rc = host_reduce(dtype, op, b + (froms[s->rank] + off) * es, ins.data(), s->p, m, s->nt);
      if (rc) return rc;
    }
    if (int rc = shm_barrier(s)) return rc;
  }
  return 0;
}

// Ragged allgather: every rank ends with every rank's [froms[j], tos[j]).
int mp4x_shm_allgather(void* h, int es, void* buf, const int64_t* froms, const int64_t* tos) {
  Shm* s = (Shm*)h;
  int64_t maxc = 0;
  for (int j = 0; j < s->p; ++j) maxc = std::max(maxc, tos[j] - froms[j]);
  const int64_t q = s->slot / es;
  char* b = (char*)buf;
  for (int64_t off = 0; off < maxc; off += q) {
    const int64_t c = tos[s->rank] - froms[s->rank];
    if (off < c) par_copy(s->slot_ptr(s->rank), b + (froms[s->rank] + off) * es, std::min(q, c - off) * es, s->nt);
    if (int rc = shm_barrier(s)) return rc;
    for (int j = 0; j < s->p; ++j) {
      const int64_t cj = tos[j] - froms[j];
      if (j != s->rank && off < cj) par_copy(b + (froms[j] + off) * es, s->slot_ptr(j), std::min(q, cj - off) * es, s->nt);
    }
    if (int rc = shm_barrier(s)) return rc;
  }
  return 0;
}

int mp4x_shm_broadcast(void* h, int es, void* buf, int64_t frm, int64_t to, int root) {
  Shm* s = (Shm*)h;
  const int64_t q = s->slot / es;
  char* b = (char*)buf;
  for (int64_t off = frm; off < to; off += q) {
    const int64_t m = std::min(q, to - off);
    if (s->rank == root) par_copy(s->slot_ptr(root), b + off * es, m * es, s->nt);
    if (int rc = shm_barrier(s)) return rc;
    if (s->rank != root) par_copy(b + off * es, s->slot_ptr(root), m * es, s->nt);
    if (int rc = shm_barrier(s)) return rc;
  }
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------- in-process thread barrier
// ThreadCommSlave's threads meet 3-4 times per collective.  Python's threading.Barrier hands a
// Condition lock around (~11 us per meeting); this sense-counting barrier spins briefly with
// `pause` and then yields (2.2 us per meeting for 2 threads), and ctypes releases the GIL for
// the whole wait.  The spin must stay SHORT: with 4096 pauses (~140 cycles each on recent Xeons)
// the meeting cost rose to 67 us, because the spinners kept the cores the GIL holder needed.
struct alignas(64) TBarrier {
  std::atomic<uint32_t> count{0};
  std::atomic<uint32_t> gen{0};
  std::atomic<uint32_t> abort{0};
  std::atomic<uint32_t> sleepers{0};
  uint32_t n;
  double timeout_s;
  BarrierWords words() { return BarrierWords{&count, &gen, &abort, &sleepers, n, timeout_s, false}; }
};

extern "C" void* mp4x_tbarrier_create(int n, double timeout_s) {
  if (n < 1) return nullptr;
  TBarrier* b = new TBarrier();
  b->n = (uint32_t)n;
  b->timeout_s = timeout_s > 0 ? timeout_s : 1e30;
  return b;
}

extern "C" void mp4x_tbarrier_destroy(void* h) { delete (TBarrier*)h; }

extern "C" void mp4x_tbarrier_abort(void* h) {
  TBarrier* b = (TBarrier*)h;
  b->abort.store(1, std::memory_order_seq_cst);
  futex_op(&b->gen, FUTEX_WAKE, INT_MAX, nullptr, false);   // sleepers re-check `abort`
}

extern "C" int mp4x_tbarrier_aborted(void* h) { return (int)((TBarrier*)h)->abort.load(std::memory_order_acquire); }

// 0: released; -1: timed out (the barrier is then aborted for everyone); -2: aborted.
extern "C" int mp4x_tbarrier_wait(void* h) {
  TBarrier* b = (TBarrier*)h;
  return barrier_wait(b->words());
}

// ---------------------------------------------------------------- native thread-team collectives
// The thread level of ThreadCommSlave for host arrays, entirely below the GIL: every thread
// makes ONE call per phase; the rendezvous, the data-parallel chunked reduction (thread t
// reduces chunk t of [f, t) over all T buffers, the root thread's value first, then the others
// in thread order — the reference's thread reduce, ThreadCommSlave.java:259-303) and the
// copy-back all run in C++.  Python pays one GIL release/re-acquire per phase instead of one
// per barrier.
//
// GIL hand-off.  When a collective returns, every thread wants the GIL at once: all but one
// sleep on CPython's GIL condition variable and are woken by a futex when the holder next
// releases it -- that wake-up, not the data movement, used to dominate a small call (~20 us of
// BASELINE config 1's 2-thread float[1024] allreduce).  So the threads leave in a chain: thread
// 0 returns at once; thread t keeps spinning HERE (GIL still released) until thread t-1 has
// entered its next team call -- ctypes released the GIL before that entry -- and only then
// returns, to find the GIL free.  The threads' Python then runs back to back with no sleeping
// hand-off.  The spin is bounded (MP4X_TEAM_HANDOFF_US, default 30; 0 turns it off), so a peer
// that does other work between calls costs at most that much spinning, never a hang.
struct Team {
  TBarrier bar;
  std::vector<void*> slots;
  std::unique_ptr<std::atomic<uint64_t>[]> entered;   // team calls entered, per thread
  double handoff_s = 30e-6;
};

extern "C" void* mp4x_team_create(int n, double timeout_s) {
  if (n < 1) return nullptr;
  Team* t = new Team();
  t->bar.n = (uint32_t)n;
  t->bar.timeout_s = timeout_s > 0 ? timeout_s : 1e30;
  t->slots.assign(n, nullptr);
  t->entered.reset(new std::atomic<uint64_t>[n]);
  for (int i = 0; i < n; ++i) t->entered[i].store(0, std::memory_order_relaxed);
  if (const char* e = std::getenv("MP4X_TEAM_HANDOFF_US")) t->handoff_s = std::atof(e) * 1e-6;
  return t;
}

// Every team call starts here: count the entry (what thread tid+1's team_leave waits for).
static inline uint64_t team_enter(Team* tm, int tid) {
  return tm->entered[tid].fetch_add(1, std::memory_order_acq_rel) + 1;
}

// Every team call ends here: `k` is this call's sequence number (team calls are collective, so
// thread tid-1's k-th call is the same collective); wait, bounded, for its (k+1)-th.
static inline int team_leave(Team* tm, int tid, uint64_t k, int rc) {
  if (rc || tid == 0 || tm->handoff_s <= 0) return rc;
  const std::atomic<uint64_t>& prev = tm->entered[tid - 1];
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 1; prev.load(std::memory_order_acquire) <= k; ++i) {
    if (tm->bar.abort.load(std::memory_order_relaxed)) break;
    __builtin_ia32_pause();
    if ((i & 31) == 0) {
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > tm->handoff_s) break;
      // if the scheduler put the GIL holder on THIS cpu, spinning would only delay it
      if ((i & 255) == 0) sched_yield();
    }
  }
  return rc;
}

extern "C" void mp4x_team_destroy(void* h) { delete (Team*)h; }
extern "C" int mp4x_team_barrier(void* h, int tid) {
  Team* tm = (Team*)h;
  const uint64_t k = team_enter(tm, tid);
  return team_leave(tm, tid, k, mp4x_tbarrier_wait(&tm->bar));
}
extern "C" int mp4x_team_aborted(void* h) { return mp4x_tbarrier_aborted(&((Team*)h)->bar); }
extern "C" void mp4x_team_abort(void* h) { mp4x_tbarrier_abort(&((Team*)h)->bar); }

static inline void team_chunk(int64_t f, int64_t t, int T, int tid, int64_t* lo, int64_t* hi) {
  const int64_t n = t - f;
  *lo = f + n * tid / T;
  *hi = f + n * (tid + 1) / T;
}

// Thread tid's chunk of [f, t): all T buffers reduced into the root's (root's value first, then
// the others in thread order); with `spread`, the result also copied into every other buffer's
// chunk (the chunks are disjoint, so that needs no extra barrier).
static int team_reduce_chunk(Team* tm, int tid, int64_t f, int64_t t, int dtype, int op, int root, bool spread) {
  const int T = (int)tm->bar.n;
  const int es = esize(dtype);
  int64_t lo, hi;
  team_chunk(f, t, T, tid, &lo, &hi);
  if (hi <= lo) return 0;
  const void* ins[64];
  std::vector<const void*> big;
  const void** in = ins;
  if (T > 64) {
    big.resize(T);
    in = big.data();
  }
  int m = 0;
  in[m++] = (const char*)tm->slots[root] + lo * es;
  for (int j = 0; j < T; ++j)
    if (j != root) in[m++] = (const char*)tm->slots[j] + lo * es;
  char* out = (char*)tm->slots[root] + lo * es;
  if (int rc = host_reduce(dtype, op, out, in, T, hi - lo, 1)) return rc;
  if (spread)
    for (int j = 0; j < T; ++j)
      if (j != root) std::memcpy((char*)tm->slots[j] + lo * es, out, (hi - lo) * es);
  return 0;
}

static int team_reduce_phase(Team* tm, int tid, void* buf, int64_t f, int64_t t, int dtype, int op, int root,
                             bool spread) {
  tm->slots[tid] = buf;
  if (int rc = mp4x_tbarrier_wait(&tm->bar)) return rc;
  if (int rc = team_reduce_chunk(tm, tid, f, t, dtype, op, root, spread)) {
    mp4x_tbarrier_abort(&tm->bar);
    return rc;
  }
  return mp4x_tbarrier_wait(&tm->bar);
}

// [f, t) of every thread's buffer reduced into the root thread's buffer (then a barrier).
extern "C" int mp4x_team_reduce(void* h, int tid, void* buf, int64_t f, int64_t t, int dtype, int op, int root) {
  if (!esize(dtype)) return MP4X_E_UNSUPPORTED;
  Team* tm = (Team*)h;
  const uint64_t k = team_enter(tm, tid);
  return team_leave(tm, tid, k, team_reduce_phase(tm, tid, buf, f, t, dtype, op, root, false));
}

// Root's [f, t) copied into every other thread's buffer: publish, barrier, copy, barrier.
extern "C" int mp4x_team_bcast(void* h, int tid, void* buf, int64_t f, int64_t t, int elem_bytes, int root) {
  Team* tm = (Team*)h;
  const uint64_t k = team_enter(tm, tid);
  tm->slots[tid] = buf;
  int rc = mp4x_tbarrier_wait(&tm->bar);
  if (!rc) {
    if (tid != root && t > f)
      std::memcpy((char*)buf + f * elem_bytes, (const char*)tm->slots[root] + f * elem_bytes, (t - f) * elem_bytes);
    rc = mp4x_tbarrier_wait(&tm->bar);
  }
  return team_leave(tm, tid, k, rc);
}

// Fused thread-level allreduce (slaveNum == 1): publish, barrier, each thread reduces its chunk
// of every buffer and writes the result into every buffer's chunk, barrier.  Two meetings.
extern "C" int mp4x_team_allreduce(void* h, int tid, void* buf, int64_t f, int64_t t, int dtype, int op) {
  if (!esize(dtype)) return MP4X_E_UNSUPPORTED;
  Team* tm = (Team*)h;
  const uint64_t k = team_enter(tm, tid);
  return team_leave(tm, tid, k, team_reduce_phase(tm, tid, buf, f, t, dtype, op, 0, true));
}
