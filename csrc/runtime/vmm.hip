// Library-owned device allocations that can be mapped into every peer at ANY size (the
// ncclMemAlloc analogue of mp4x, ``ProcessCommSlave.memAlloc``).
//
// Why: hipIpcGetMemHandle/hipIpcOpenMemHandle maps a whole hipMalloc allocation, and on this
// ROCm an open of an allocation of 2^31 bytes or more never returns
// (profiles/r2/ipc_open_probe.jsonl).  The reference allreduces 8 GB arrays in place
// (/root/reference/README.md:313, ProcessCommSlave.java:1733-1763); the zero-copy kernels need
// those tensors mapped in every peer.  So the allocation is built from the virtual memory API:
//
//   * physical chunks (hipMemCreate, ``chunk`` bytes each, a granularity multiple well below
//     2 GiB) are mapped back to back into ONE reserved VA range: the tensor is contiguous;
//   * every chunk is exported as a POSIX file descriptor (dmabuf) — the fds travel to the
//     same-node peers over a unix socket (SCM_RIGHTS, parallel/vmm.py);
//   * a peer imports every fd, maps the chunks back to back into its own reserved VA range
//     and grants its device read/write access: one contiguous peer view of the whole tensor,
//     so the zero-copy kernels (ipc.hip) run on it unchanged.
//
// Memory is coarse-grained device memory (like hipMalloc), which is what the zero-copy kernels
// already run on for registered caching-allocator tensors.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <unistd.h>

namespace {

hipMemAllocationProp make_prop(int dev) {
  hipMemAllocationProp prop;
  std::memset(&prop, 0, sizeof(prop));
  prop.type = hipMemAllocationTypePinned;
  prop.requestedHandleTypes = hipMemHandleTypePosixFileDescriptor;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  return prop;
}

// VA alignment of a reservation: 2 MiB (large-fragment friendly) when the chunk size is a 2 MiB
// multiple, else the runtime default (the alignment must be a power of two; a chunk size in
// general is not).
size_t va_alignment(size_t chunk) { return chunk % (2u << 20) == 0 ? (2u << 20) : 0; }

// Address hint mode (MP4X_VMM_POLICY=hint, an A/B of the memFree lifetime study): every new
// reservation asks for the address above the highest range reserved so far, so a range freed
// earlier is never handed out again while its physical memory does go back to the device.
bool g_hint_on = false;
uintptr_t g_cursor = 0;

hipError_t reserve(void** va, size_t total, size_t align) {
  void* want = (g_hint_on && g_cursor) ? reinterpret_cast<void*>(g_cursor) : nullptr;
  hipError_t e = hipMemAddressReserve(va, total, align, want, 0);
  if (e == hipSuccess && g_hint_on) {
    const uintptr_t end = reinterpret_cast<uintptr_t>(*va) + total + (4u << 20);   // a 4 MiB gap
    const uintptr_t next = (end + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
    if (next > g_cursor) g_cursor = next;
  }
  return e;
}

hipError_t grant(void* va, size_t bytes, int dev) {
  hipMemAccessDesc acc;
  std::memset(&acc, 0, sizeof(acc));
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = dev;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  return hipMemSetAccess(va, bytes, &acc, 1);
}

// unmap + release chunks [0, n) and free the VA range (best effort, first error returned)
int teardown(void* va, size_t chunk, int n, const uint64_t* handles, size_t reserved) {
  int first = 0;
  for (int i = 0; i < n; ++i) {
    if (va) {
      hipError_t e = hipMemUnmap(static_cast<char*>(va) + (size_t)i * chunk, chunk);
      if (e != hipSuccess && !first) first = (int)e;
    }
    if (handles[i]) {
      hipError_t e = hipMemRelease((hipMemGenericAllocationHandle_t)(uintptr_t)handles[i]);
      if (e != hipSuccess && !first) first = (int)e;
    }
  }
  if (va && reserved) {
    hipError_t e = hipMemAddressFree(va, reserved);
    if (e != hipSuccess && !first) first = (int)e;
  }
  return first;
}

}  // namespace

// Recommended allocation granularity (bytes) of the current device for fd-exportable memory.
extern "C" int mp4x_vmm_granularity(size_t* gran) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  hipMemAllocationProp prop = make_prop(dev);
  return (int)hipMemGetAllocationGranularity(gran, &prop, hipMemAllocationGranularityRecommended);
}

// Allocate ``n`` chunks of ``chunk`` bytes (granularity multiple) mapped back to back at a
// fresh VA range.  ``fds`` (n entries) get one exported POSIX fd per chunk when ``fds`` is not
// null; ``handles`` (n entries) get the generic allocation handles.  On failure everything
// created so far is released and the fds closed.
extern "C" int mp4x_vmm_create(size_t chunk, int n, void** va_out, uint64_t* handles, int* fds) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  const size_t total = chunk * (size_t)n;
  for (int i = 0; i < n; ++i) {
    handles[i] = 0;
    if (fds) fds[i] = -1;
  }
  void* va = nullptr;
  e = reserve(&va, total, va_alignment(chunk));
  if (e != hipSuccess) return (int)e;
  hipMemAllocationProp prop = make_prop(dev);
  int mapped = 0;
  for (int i = 0; i < n && e == hipSuccess; ++i) {
    hipMemGenericAllocationHandle_t h;
    e = hipMemCreate(&h, chunk, &prop, 0);
    if (e != hipSuccess) break;
    handles[i] = (uint64_t)(uintptr_t)h;
    e = hipMemMap(static_cast<char*>(va) + (size_t)i * chunk, chunk, 0, h, 0);
    if (e != hipSuccess) break;
    mapped = i + 1;
    if (fds) {
      int fd = -1;
      e = hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0);
      if (e != hipSuccess) break;
      fds[i] = fd;
    }
  }
  if (e == hipSuccess) e = grant(va, total, dev);
  if (e != hipSuccess) {
    if (fds)
      for (int i = 0; i < n; ++i)
        if (fds[i] >= 0) { close(fds[i]); fds[i] = -1; }
    // chunks [mapped, n) were created but not mapped: release them without unmapping
    for (int i = 0; i < mapped; ++i) hipMemUnmap(static_cast<char*>(va) + (size_t)i * chunk, chunk);
    for (int i = 0; i < n; ++i)
      if (handles[i]) { hipMemRelease((hipMemGenericAllocationHandle_t)(uintptr_t)handles[i]); handles[i] = 0; }
    hipMemAddressFree(va, total);
    return (int)e;
  }
  *va_out = va;
  return 0;
}

// Import a peer's ``n`` chunk fds and map them back to back at a fresh VA range of this
// process, read/write for the current device.  The fds are NOT closed here (the caller owns
// them; the imported handles keep the memory alive).
extern "C" int mp4x_vmm_import(const int* fds, size_t chunk, int n, void** va_out, uint64_t* handles) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  const size_t total = chunk * (size_t)n;
  for (int i = 0; i < n; ++i) handles[i] = 0;
  void* va = nullptr;
  e = reserve(&va, total, va_alignment(chunk));
  if (e != hipSuccess) return (int)e;
  int mapped = 0;
  for (int i = 0; i < n && e == hipSuccess; ++i) {
    hipMemGenericAllocationHandle_t h;
    // HIP reads the POSIX fd THROUGH the osHandle pointer (passing the fd value itself, the
    // CUDA convention, makes the runtime dereference a small integer: measured SIGSEGV on
    // ROCm 7 / gfx950, tools/vmm_probe.py)
    int fd = fds[i];
    e = hipMemImportFromShareableHandle(&h, static_cast<void*>(&fd), hipMemHandleTypePosixFileDescriptor);
    if (e != hipSuccess) break;
    handles[i] = (uint64_t)(uintptr_t)h;
    e = hipMemMap(static_cast<char*>(va) + (size_t)i * chunk, chunk, 0, h, 0);
    if (e == hipSuccess) mapped = i + 1;
  }
  if (e == hipSuccess) e = grant(va, total, dev);
  if (e != hipSuccess) {
    for (int i = 0; i < mapped; ++i) hipMemUnmap(static_cast<char*>(va) + (size_t)i * chunk, chunk);
    for (int i = 0; i < n; ++i)
      if (handles[i]) { hipMemRelease((hipMemGenericAllocationHandle_t)(uintptr_t)handles[i]); handles[i] = 0; }
    hipMemAddressFree(va, total);
    return (int)e;
  }
  *va_out = va;
  return 0;
}

// Unmap + release ``n`` chunks mapped at ``va`` and free the VA range (own or imported).
extern "C" int mp4x_vmm_free(void* va, size_t chunk, int n, const uint64_t* handles) {
  return teardown(va, chunk, n, handles, chunk * (size_t)n);
}

// Unmap + release the chunks but keep the VA range reserved for the rest of the process: no
// later reservation lands on these addresses, and no hipMemAddressFree happens (see the chunk
// pool below for why).  MP4X_VMM_POLICY fresh_va / keep_*_va, parallel/ipc.py mem_free.
extern "C" int mp4x_vmm_release_keep_va(void* va, size_t chunk, int n, const uint64_t* handles) {
  return teardown(va, chunk, n, handles, 0);
}

// ---------------------------------------------------------------- chunk pool (memAlloc default)
// On the HIP runtime PyTorch-ROCm ships, (a) hipMemRelease of an exported chunk never gives the
// memory back to the device, and (b) once a process has called hipMemAddressFree on a range it
// had mapped, the chunks it exports LATER read as other memory in the importers — shown with
// plain HIP in tools/repro/ipc_lifetime_repro.hip (profiles/r4/lifetime/).  So memAlloc keeps
// physical chunks for reuse (parallel/vmm.py ChunkPool) and never frees a VA range: an allocation
// maps pooled chunks into a fresh range, memFree only unmaps.

// One physical chunk of ``bytes`` (granularity multiple); ``fd`` (nullable) gets its dmabuf fd.
extern "C" int mp4x_vmm_chunk_create(size_t bytes, uint64_t* handle, int* fd) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  hipMemAllocationProp prop = make_prop(dev);
  hipMemGenericAllocationHandle_t h;
  e = hipMemCreate(&h, bytes, &prop, 0);
  if (e != hipSuccess) return (int)e;
  if (fd) {
    *fd = -1;
    e = hipMemExportToShareableHandle(fd, h, hipMemHandleTypePosixFileDescriptor, 0);
    if (e != hipSuccess) {
      hipMemRelease(h);
      return (int)e;
    }
  }
  *handle = (uint64_t)(uintptr_t)h;
  return 0;
}

// A peer's chunk from its dmabuf fd (the fd stays the caller's).
extern "C" int mp4x_vmm_chunk_import(int fd, uint64_t* handle) {
  hipMemGenericAllocationHandle_t h;
  int v = fd;     // read THROUGH the pointer by this runtime (see mp4x_vmm_import)
  hipError_t e = hipMemImportFromShareableHandle(&h, static_cast<void*>(&v), hipMemHandleTypePosixFileDescriptor);
  if (e != hipSuccess) return (int)e;
  *handle = (uint64_t)(uintptr_t)h;
  return 0;
}

extern "C" int mp4x_vmm_chunk_release(uint64_t handle) {
  return (int)hipMemRelease((hipMemGenericAllocationHandle_t)(uintptr_t)handle);
}

// Reserve a fresh range of sum(sizes) bytes and map ``n`` chunks back to back, read/write for the
// current device.  On failure the chunks mapped so far are unmapped and the range is left
// reserved (never freed, see above); *va_out gets it either way (0 if the reservation failed).
extern "C" int mp4x_vmm_map_chunks(const uint64_t* handles, const size_t* sizes, int n, void** va_out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  size_t total = 0;
  bool big = true;
  for (int i = 0; i < n; ++i) {
    total += sizes[i];
    big = big && sizes[i] % (2u << 20) == 0;
  }
  void* va = nullptr;
  *va_out = nullptr;
  e = reserve(&va, total, big ? (2u << 20) : 0);
  if (e != hipSuccess) return (int)e;
  *va_out = va;
  size_t off = 0;
  int mapped = 0;
  for (int i = 0; i < n && e == hipSuccess; ++i) {
    e = hipMemMap(static_cast<char*>(va) + off, sizes[i], 0, (hipMemGenericAllocationHandle_t)(uintptr_t)handles[i], 0);
    if (e == hipSuccess) {
      off += sizes[i];
      mapped = i + 1;
    }
  }
  if (e == hipSuccess) e = grant(va, total, dev);
  if (e != hipSuccess) {
    off = 0;
    for (int i = 0; i < mapped; ++i) {
      hipMemUnmap(static_cast<char*>(va) + off, sizes[i]);
      off += sizes[i];
    }
  }
  return (int)e;
}

// Unmap ``n`` chunks mapped back to back at ``va`` (the range stays reserved, the chunks alive).
extern "C" int mp4x_vmm_unmap_chunks(void* va, const size_t* sizes, int n) {
  int first = 0;
  size_t off = 0;
  for (int i = 0; i < n; ++i) {
    hipError_t e = hipMemUnmap(static_cast<char*>(va) + off, sizes[i]);
    if (e != hipSuccess && !first) first = (int)e;
    off += sizes[i];
  }
  return first;
}

// Turn the address hint mode on / off; returns the cursor (the next hinted address, 0 = none yet).
extern "C" uint64_t mp4x_vmm_va_hint(int on) {
  g_hint_on = on != 0;
  return (uint64_t)g_cursor;
}

// System-scope release on every XCD: each workgroup's lane 0 issues a release fence at system
// scope (L2 write-back of that XCD's dirty lines), with enough workgroups that every XCD runs
// several of them.  Makes what earlier kernels wrote into coarse-grained memory visible to
// readers that do not go through this GPU's L2 (a peer over xGMI, or another mapping).
__global__ void __launch_bounds__(64) k_release_all_xcds() {
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

extern "C" int mp4x_release_all(void* stream) {
  hipLaunchKernelGGL(k_release_all_xcds, dim3(1024), dim3(64), 0, static_cast<hipStream_t>(stream));
  return (int)hipGetLastError();
}
