// Experiment: the library's own K6b encode on an all-zero 256 MiB input (WRITE_SIZE check).
#include "../../csrc/kernels/codec.hip"

int main(int argc, char** argv) {
  const int64_t n = 64ll << 20, nblk = n / 256;
  const float density = argc > 1 ? atof(argv[1]) : 0.0f;
  uint32_t *in, *vals;
  int64_t *offs, *table;
  uint64_t* masks;
  int32_t* counts;
  hipMalloc(&in, n * 4);
  hipMalloc(&vals, n * 4);
  hipMalloc(&offs, (nblk + 1) * 8);
  hipMalloc(&masks, nblk * 32);
  hipMalloc(&counts, nblk * 4);
  hipMalloc(&table, 4 * 8);
  hipMemset(in, 0, n * 4);
  if (density > 0) {   // every 1/density-th word non-zero
    const int stride = (int)(1.0f / density);
    uint32_t* h = (uint32_t*)malloc(n * 4);
    for (int64_t i = 0; i < n; ++i) h[i] = (i % stride == 0) ? 1u : 0u;
    hipMemcpy(in, h, n * 4, hipMemcpyHostToDevice);
    free(h);
  }
  int64_t ht[4] = {0, n, 0, nblk};
  hipMemcpy(table, ht, sizeof(ht), hipMemcpyHostToDevice);
  size_t tb = mp4x_zs_temp_bytes(nblk);
  void* temp;
  hipMalloc(&temp, tb);
  hipDeviceSynchronize();
  for (int rep = 0; rep < 2; ++rep) {
    int e = mp4x_zs_encode(4, in, table, 1, nblk, masks, counts, offs, vals, temp, tb, nullptr);
    if (e) { printf("encode error %d\n", e); return 1; }
  }
  hipError_t e = hipDeviceSynchronize();
  int64_t total = 0;
  hipMemcpy(&total, offs + nblk, 8, hipMemcpyDeviceToHost);
  printf("done %d total=%lld\n", (int)e, (long long)total);
  return (int)e;
}
