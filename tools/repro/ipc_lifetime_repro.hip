// Standalone two-process reproducer of the two memory-lifetime anomalies mp4x worked around in
// rounds 2-3 (VERDICT r3 "What's weak" #4) — plain HIP, no torch, no mp4x:
//
//   ipc : exporter hipMalloc's X, writes pattern A, hipIpcGetMemHandle; importer opens it, reads,
//         closes it (hipIpcCloseMemHandle).  Exporter frees X, hipMalloc's Y of the same size
//         (usually at the recycled address), writes pattern B, exports again; importer opens the
//         new handle and reads.  Does it see B?  Variants: importer closes before / after the
//         exporter frees; importer does not close at all (the mp4x workaround).
//   vmm : exporter hipMemCreate's a chunk, maps it, writes A, exports a dmabuf fd (SCM_RIGHTS to
//         the importer); importer imports, maps at its own VA, reads.  Then both release (order
//         per variant: importer first, exporter first), the exporter creates a NEW chunk with
//         pattern B and exports it; the importer imports and reads.  Does it see B (r3 saw
//         zeros)?  Variants also keep the first import alive / keep fds open, keep the first VA
//         ranges reserved so the second mapping lands at fresh addresses (fresh_va), or let the
//         exporter import its own fd as a control (self_import).
//
// Reads go through a kernel (the path of the zero-copy collectives) and through hipMemcpy.
// Usage: ipc_lifetime_repro exporter <ipc|vmm> <variant> <name> [bytes] &
//        ipc_lifetime_repro importer <ipc|vmm> <variant> <name> [bytes]   (one JSON line per check)
// Build: hipcc --offload-arch=gfx950 -O2 -o ipc_lifetime_repro ipc_lifetime_repro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <cstddef>
#include <sys/socket.h>
#include <sys/un.h>
#include <sys/wait.h>
#include <unistd.h>

#define CK(x)                                                                                     \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      fprintf(stderr, "[%s] %s:%d %s -> %s\n", role, __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      _exit(3);                                                                                   \
    }                                                                                             \
  } while (0)

static const char* role = "main";

__global__ void k_fill(uint32_t* p, size_t n, uint32_t salt) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)(i * 2654435761u) ^ salt;
}

// reads through the mapping in a kernel (as the zero-copy collectives do): count mismatches
__global__ void k_check(const uint32_t* p, size_t n, uint32_t salt, unsigned long long* bad, uint32_t* first) {
  unsigned long long b = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t v = __builtin_nontemporal_load(p + i);
    if (v != ((uint32_t)(i * 2654435761u) ^ salt)) {
      ++b;
      if (i == 0) *first = v;
    }
  }
  if (b) atomicAdd(bad, b);
}

// ---------------------------------------------------------------- tiny message channel
static void send_msg(int s, const void* buf, size_t len, int fd = -1) {
  struct msghdr m;
  memset(&m, 0, sizeof(m));
  struct iovec io = {const_cast<void*>(buf), len};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  char cbuf[CMSG_SPACE(sizeof(int))];
  if (fd >= 0) {
    memset(cbuf, 0, sizeof(cbuf));
    m.msg_control = cbuf;
    m.msg_controllen = sizeof(cbuf);
    struct cmsghdr* c = CMSG_FIRSTHDR(&m);
    c->cmsg_level = SOL_SOCKET;
    c->cmsg_type = SCM_RIGHTS;
    c->cmsg_len = CMSG_LEN(sizeof(int));
    memcpy(CMSG_DATA(c), &fd, sizeof(int));
  }
  if (sendmsg(s, &m, 0) != (ssize_t)len) { perror("sendmsg"); _exit(4); }
}

static int recv_msg(int s, void* buf, size_t len) {   // returns a received fd or -1
  struct msghdr m;
  memset(&m, 0, sizeof(m));
  struct iovec io = {buf, len};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  char cbuf[CMSG_SPACE(sizeof(int))];
  m.msg_control = cbuf;
  m.msg_controllen = sizeof(cbuf);
  if (recvmsg(s, &m, MSG_WAITALL) != (ssize_t)len) { perror("recvmsg"); _exit(4); }
  int fd = -1;
  for (struct cmsghdr* c = CMSG_FIRSTHDR(&m); c; c = CMSG_NXTHDR(&m, c))
    if (c->cmsg_level == SOL_SOCKET && c->cmsg_type == SCM_RIGHTS) memcpy(&fd, CMSG_DATA(c), sizeof(int));
  return fd;
}

static void sync_point(int s, const char* tag) {       // both sides meet here
  char t[16] = {0};
  strncpy(t, tag, 15);
  send_msg(s, t, 16);
  char u[16];
  recv_msg(s, u, 16);
  if (strncmp(t, u, 16)) { fprintf(stderr, "[%s] sync mismatch %s / %s\n", role, t, u); _exit(5); }
}

static void check_read(const void* p, size_t n, uint32_t salt, const char* what, const char* variant, const char* mode) {
  unsigned long long* bad;
  uint32_t* first;
  CK(hipMalloc(&bad, 8));
  CK(hipMalloc(&first, 4));
  CK(hipMemset(bad, 0, 8));
  CK(hipMemset(first, 0xff, 4));
  hipLaunchKernelGGL(k_check, dim3(256), dim3(256), 0, 0, (const uint32_t*)p, n, salt, bad, first);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  unsigned long long hb = 0;
  uint32_t hf = 0;
  CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost));
  uint32_t* host = (uint32_t*)malloc(n * 4);
  CK(hipMemcpy(host, p, n * 4, hipMemcpyDeviceToHost));
  size_t cbad = 0;
  for (size_t i = 0; i < n; ++i) cbad += host[i] != ((uint32_t)(i * 2654435761u) ^ salt);
  printf("{\"mode\": \"%s\", \"variant\": \"%s\", \"check\": \"%s\", \"kernel_wrong\": %llu, \"copy_wrong\": %zu, "
         "\"n\": %zu, \"first_word\": %u, \"expect_first\": %u}\n",
         mode, variant, what, hb, cbad, n, hf == 0xffffffffu ? host[0] : hf, salt);
  fflush(stdout);
  free(host);
  CK(hipFree(bad));
  CK(hipFree(first));
}

// ---------------------------------------------------------------- hipIpc* handles
static void ipc_exporter(int s, size_t bytes, const std::string& v) {
  role = "exporter";
  CK(hipSetDevice(0));
  const size_t n = bytes / 4;
  void* x;
  CK(hipMalloc(&x, bytes));
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, (uint32_t*)x, n, 0xA0A0A0A0u);
  CK(hipDeviceSynchronize());
  hipIpcMemHandle_t h1;
  CK(hipIpcGetMemHandle(&h1, x));
  send_msg(s, &h1, sizeof(h1));
  sync_point(s, "read1");
  if (v != "close_after_free") sync_point(s, "closed1");
  CK(hipFree(x));
  void* y;
  CK(hipMalloc(&y, bytes));
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, (uint32_t*)y, n, 0xB1B1B1B1u);
  CK(hipDeviceSynchronize());
  hipIpcMemHandle_t h2;
  CK(hipIpcGetMemHandle(&h2, y));
  printf("{\"mode\": \"ipc\", \"variant\": \"%s\", \"same_address\": %d, \"same_handle_bytes\": %d}\n", v.c_str(),
         x == y, memcmp(&h1, &h2, sizeof(h1)) == 0);
  fflush(stdout);
  send_msg(s, &h2, sizeof(h2));
  sync_point(s, "read2");
  CK(hipFree(y));
}

static void ipc_importer(int s, size_t bytes, const std::string& v) {
  role = "importer";
  CK(hipSetDevice(0));
  const size_t n = bytes / 4;
  hipIpcMemHandle_t h1, h2;
  recv_msg(s, &h1, sizeof(h1));
  void* p1;
  CK(hipIpcOpenMemHandle(&p1, h1, hipIpcMemLazyEnablePeerAccess));
  check_read(p1, n, 0xA0A0A0A0u, "first", v.c_str(), "ipc");
  sync_point(s, "read1");
  if (v == "close_before_free") CK(hipIpcCloseMemHandle(p1));
  if (v != "close_after_free") sync_point(s, "closed1");
  recv_msg(s, &h2, sizeof(h2));
  if (v == "close_after_free") CK(hipIpcCloseMemHandle(p1));
  void* p2;
  CK(hipIpcOpenMemHandle(&p2, h2, hipIpcMemLazyEnablePeerAccess));
  printf("{\"mode\": \"ipc\", \"variant\": \"%s\", \"importer_same_va\": %d}\n", v.c_str(), p1 == p2);
  check_read(p2, n, 0xB1B1B1B1u, "second", v.c_str(), "ipc");
  sync_point(s, "read2");
  CK(hipIpcCloseMemHandle(p2));
  if (v == "never_close" && p1 != p2) CK(hipIpcCloseMemHandle(p1));
}

// ---------------------------------------------------------------- VMM chunks + dmabuf fds
static hipMemAllocationProp vmm_prop() {
  hipMemAllocationProp prop;
  memset(&prop, 0, sizeof(prop));
  prop.type = hipMemAllocationTypePinned;
  prop.requestedHandleTypes = hipMemHandleTypePosixFileDescriptor;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  return prop;
}

static void grant(void* va, size_t bytes) {
  hipMemAccessDesc acc;
  memset(&acc, 0, sizeof(acc));
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = 0;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(va, bytes, &acc, 1));
}

struct Region {
  void* va = nullptr;
  hipMemGenericAllocationHandle_t h{};
  size_t bytes = 0;
};

static bool g_self_import = false;   // variant self_import: the exporter imports its own fd too

static Region vmm_create(size_t bytes, uint32_t salt, int* fd) {
  Region r;
  r.bytes = bytes;
  hipMemAllocationProp prop = vmm_prop();
  CK(hipMemAddressReserve(&r.va, bytes, 2u << 20, nullptr, 0));
  CK(hipMemCreate(&r.h, bytes, &prop, 0));
  CK(hipMemMap(r.va, bytes, 0, r.h, 0));
  grant(r.va, bytes);
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, (uint32_t*)r.va, bytes / 4, salt);
  CK(hipDeviceSynchronize());
  CK(hipMemExportToShareableHandle(fd, r.h, hipMemHandleTypePosixFileDescriptor, 0));
  if (!g_self_import) return r;
  // control: can THIS process import its own fd?
  hipMemGenericAllocationHandle_t hs{};
  int dup_fd = *fd;
  const hipError_t es = hipMemImportFromShareableHandle(&hs, (void*)&dup_fd, hipMemHandleTypePosixFileDescriptor);
  printf("{\"mode\": \"vmm\", \"self_import\": \"%s\", \"fd\": %d, \"fd_size\": %lld}\n", hipGetErrorString(es),
         *fd, (long long)lseek(*fd, 0, SEEK_END));
  fflush(stdout);
  lseek(*fd, 0, SEEK_SET);
  if (es == hipSuccess) CK(hipMemRelease(hs));
  return r;
}

static Region vmm_import(int fd, size_t bytes) {
  Region r;
  r.bytes = bytes;
  // HIP reads the fd THROUGH the handle pointer (tools/vmm_probe.py)
  hipError_t e = hipMemImportFromShareableHandle(&r.h, (void*)&fd, hipMemHandleTypePosixFileDescriptor);
  if (e != hipSuccess) {   // say what the fd is before giving up
    char link[256] = {0}, path[64];
    snprintf(path, sizeof(path), "/proc/self/fd/%d", fd);
    ssize_t k = readlink(path, link, sizeof(link) - 1);
    const off_t sz = fd >= 0 ? lseek(fd, 0, SEEK_END) : -1;
    printf("{\"mode\": \"vmm\", \"import_error\": \"%s\", \"fd\": %d, \"fd_target\": \"%s\", \"fd_size\": %lld}\n",
           hipGetErrorString(e), fd, k > 0 ? link : "?", (long long)sz);
    fflush(stdout);
    _exit(3);
  }
  CK(hipMemAddressReserve(&r.va, bytes, 2u << 20, nullptr, 0));
  CK(hipMemMap(r.va, bytes, 0, r.h, 0));
  grant(r.va, bytes);
  return r;
}

// keep_va: unmap + release the physical chunk but keep the VA range reserved (freed at exit), so
// the next reservation cannot land on the same addresses (variant fresh_va)
static void vmm_free(Region& r, bool keep_va = false) {
  CK(hipDeviceSynchronize());
  CK(hipMemUnmap(r.va, r.bytes));
  CK(hipMemRelease(r.h));
  if (!keep_va) CK(hipMemAddressFree(r.va, r.bytes));
  r.h = hipMemGenericAllocationHandle_t{};
  if (!keep_va) r = Region();
}

static void vmm_exporter(int s, size_t bytes, const std::string& v) {
  role = "exporter";
  g_self_import = v == "self_import";
  CK(hipSetDevice(0));
  int fd1 = -1;
  Region a = vmm_create(bytes, 0xA0A0A0A0u, &fd1);
  char z[8] = {0};
  send_msg(s, z, 8, fd1);
  if (v != "keep_fds") close(fd1);
  sync_point(s, "read1");
  if (v == "importer_first" || v == "keep_fds" || v == "fresh_va" || v == "self_import") sync_point(s, "imp_released");
  if (v != "exporter_keeps") vmm_free(a, v == "fresh_va");
  if (v == "exporter_first") sync_point(s, "exp_released");
  int fd2 = -1;
  Region b = vmm_create(bytes, 0xB1B1B1B1u, &fd2);
  printf("{\"mode\": \"vmm\", \"variant\": \"%s\", \"fd1\": %d, \"fd2\": %d, \"same_handle\": %d}\n", v.c_str(), fd1, fd2,
         (void*)a.h == (void*)b.h);
  fflush(stdout);
  send_msg(s, z, 8, fd2);
  if (v != "keep_fds") close(fd2);
  sync_point(s, "read2");
  printf("{\"mode\": \"vmm\", \"variant\": \"%s\", \"exporter_same_va\": %d}\n", v.c_str(), a.va == b.va);
  fflush(stdout);
  vmm_free(b);
  if (v == "exporter_keeps") vmm_free(a);
  if (v == "fresh_va") CK(hipMemAddressFree(a.va, a.bytes));
}

static void vmm_importer(int s, size_t bytes, const std::string& v) {
  role = "importer";
  CK(hipSetDevice(0));
  void* warm = nullptr;                        // the runtime fully up before the first import
  CK(hipMalloc(&warm, 4096));
  CK(hipFree(warm));
  char z[8];
  int fd1 = recv_msg(s, z, 8);
  Region a = vmm_import(fd1, bytes);
  if (v != "keep_fds") close(fd1);
  check_read(a.va, bytes / 4, 0xA0A0A0A0u, "first", v.c_str(), "vmm");
  sync_point(s, "read1");
  const bool keep_import = v == "importer_keeps";
  void* const va1 = a.va;
  if (!keep_import && v != "exporter_first") vmm_free(a, v == "fresh_va");
  if (v == "importer_first" || v == "keep_fds" || v == "fresh_va" || v == "self_import") sync_point(s, "imp_released");
  if (v == "exporter_first") {
    sync_point(s, "exp_released");
    vmm_free(a);
  }
  int fd2 = recv_msg(s, z, 8);
  Region b = vmm_import(fd2, bytes);
  printf("{\"mode\": \"vmm\", \"variant\": \"%s\", \"importer_fd1\": %d, \"importer_fd2\": %d, \"importer_same_va\": %d}\n",
         v.c_str(), fd1, fd2, va1 == b.va);
  if (v != "keep_fds") close(fd2);
  check_read(b.va, bytes / 4, 0xB1B1B1B1u, "second", v.c_str(), "vmm");
  sync_point(s, "read2");
  vmm_free(b);
  if (keep_import) vmm_free(a);
  if (v == "fresh_va") CK(hipMemAddressFree(a.va, a.bytes));
}

// Two independent processes (started by the caller, e.g. tools/gpu/r4_repro.sh), each
// initialising its own HIP runtime as the ranks of a job do, meet on an abstract unix socket
// (the same channel mp4x's memAlloc uses for its fds).  No fork / exec in this program.
static int connect_pair(const std::string& name, bool server) {
  int s = socket(AF_UNIX, SOCK_STREAM, 0);
  if (s < 0) { perror("socket"); _exit(4); }
  struct sockaddr_un a;
  memset(&a, 0, sizeof(a));
  a.sun_family = AF_UNIX;
  const std::string path = "mp4x_repro_" + name;          // abstract namespace: leading NUL
  memcpy(a.sun_path + 1, path.data(), path.size());
  const socklen_t len = (socklen_t)(offsetof(struct sockaddr_un, sun_path) + 1 + path.size());
  if (server) {
    if (bind(s, (struct sockaddr*)&a, len) || listen(s, 1)) { perror("bind/listen"); _exit(4); }
    int c = accept(s, nullptr, nullptr);
    if (c < 0) { perror("accept"); _exit(4); }
    close(s);
    return c;
  }
  for (int i = 0; i < 200; ++i) {                          // the exporter may not listen yet
    if (connect(s, (struct sockaddr*)&a, len) == 0) return s;
    usleep(50000);
  }
  perror("connect");
  _exit(4);
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s <exporter|importer> <ipc|vmm> <variant> <socket name> [bytes]\n", argv[0]);
    return 2;
  }
  const std::string r = argv[1], mode = argv[2], v = argv[3];
  const size_t bytes = argc > 5 ? strtoull(argv[5], nullptr, 10) : (8u << 20);
  alarm(120);
  const int s = connect_pair(argv[4], r == "exporter");
  if (r == "exporter") {
    if (mode == "ipc") ipc_exporter(s, bytes, v);
    else vmm_exporter(s, bytes, v);
  } else {
    if (mode == "ipc") ipc_importer(s, bytes, v);
    else vmm_importer(s, bytes, v);
  }
  return 0;
}
