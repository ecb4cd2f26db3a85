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
#include <thread>
#include <type_traits>
#include <vector>

#include <sched.h>

#include "mp4x/ops.h"

namespace {

// Fork-safe fan-out (no OpenMP runtime state survives a fork in the rank launchers, and
// torch ships its own libgomp): split [0, nb) over nt threads, the caller runs chunk 0.
template <typename F>
void parallel_for(int64_t nb, int nt, F&& body) {
  if (nt <= 1 || nb <= 1) {
    for (int64_t b = 0; b < nb; ++b) body(b);
    return;
  }
  if (nt > nb) nt = (int)nb;
  std::vector<std::thread> th;
  th.reserve(nt - 1);
  auto run = [&](int t) {
    const int64_t lo = nb * t / nt, hi = nb * (t + 1) / nt;
    for (int64_t b = lo; b < hi; ++b) body(b);
  };
  for (int t = 1; t < nt; ++t) th.emplace_back(run, t);
  run(0);
  for (auto& x : th) x.join();
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

// ---------------------------------------------------------------- shared-memory engine
struct alignas(64) ShmHeader {
  std::atomic<uint32_t> count;
  std::atomic<uint32_t> gen;
  std::atomic<uint32_t> abort;
  uint32_t p;
  int64_t slot_bytes;
};
static_assert(sizeof(ShmHeader) <= 4096, "header");
static_assert(std::atomic<uint32_t>::is_always_lock_free, "process-shared atomics need lock-free");

struct Shm {
  char* base;
  ShmHeader* hdr;
  int rank, p;
  int64_t slot;
  int nt;
  double timeout_s;
  char* slot_ptr(int r) const { return base + 4096 + (int64_t)r * slot; }
};

int shm_barrier(Shm* s) {
  ShmHeader* h = s->hdr;
  const uint32_t g = h->gen.load(std::memory_order_acquire);
  if (h->count.fetch_add(1, std::memory_order_acq_rel) == (uint32_t)s->p - 1) {
    h->count.store(0, std::memory_order_relaxed);
    h->gen.fetch_add(1, std::memory_order_release);
    return 0;
  }
  auto t0 = std::chrono::steady_clock::now();
  uint64_t spins = 0;
  while (h->gen.load(std::memory_order_acquire) == g) {
    if (h->abort.load(std::memory_order_relaxed)) return -2;
    if (++spins < 256) {
      __builtin_ia32_pause();           // short waits: stay on core
    } else {
      sched_yield();                    // long waits: give the core back
      if ((spins & 1023) == 0) {
        double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el > s->timeout_s) {
          h->abort.store(1, std::memory_order_relaxed);
          return -1;
        }
      }
    }
  }
  return 0;
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
  return s;
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
