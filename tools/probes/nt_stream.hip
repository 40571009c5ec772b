// Streaming-read probe: how fast can one pass read a buffer far larger than the Infinity Cache,
// with the buffer-load cache policy as the variable (aux 0 = default, 2 = nt, 1 = sc0, 3 = sc0 nt).
// Each wave reads whole 8 KB rows (d = 1000 fp64 rows are 8000 B) with R rows in flight, the shape of
// grad_dense_multi's row loop; a checksum keeps the loads live.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/nt_stream tools/probes/nt_stream.hip && /tmp/nt_stream [GB]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

template <int AUX, int INFL>
__global__ void __launch_bounds__(256) stream_rows(const double* __restrict__ X, long long nrows, int rowbytes,
                                                   int rows_per_wave, double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const long long wave = (static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const long long r0 = wave * rows_per_wave;
  const long long r1 = r0 + rows_per_wave < nrows ? r0 + rows_per_wave : nrows;
  double acc = 0.0;
  constexpr int NV = 8;  // 8 x 16 B per lane = 8 KB per wave-row
  for (long long r = r0; r < r1; r += INFL) {
    double2 v[INFL][NV];
#pragma unroll
    for (int k = 0; k < INFL; ++k) {
      const long long rr = r + k < r1 ? r + k : r1 - 1;
      __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<char*>(reinterpret_cast<const char*>(X) + rr * rowbytes), 0, rowbytes, 0x00020000);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, (j * 64 + lane) * 16, 0, AUX);
        v[k][j] = __builtin_bit_cast(double2, q);
      }
    }
#pragma unroll
    for (int k = 0; k < INFL; ++k)
#pragma unroll
      for (int j = 0; j < NV; ++j) acc += v[k][j].x + v[k][j].y;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int AUX, int INFL>
float run(const double* X, long long nrows, int rowbytes, int rpw, double* out, int reps) {
  const long long waves = (nrows + rpw - 1) / rpw;
  const int blocks = static_cast<int>((waves + 3) / 4);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((stream_rows<AUX, INFL>), dim3(blocks), dim3(256), 0, 0, X, nrows, rowbytes, rpw, out);
  std::vector<float> ms;
  for (int i = 0; i < reps; ++i) {
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL((stream_rows<AUX, INFL>), dim3(blocks), dim3(256), 0, 0, X, nrows, rowbytes, rpw, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float t;
    CHECK(hipEventElapsedTime(&t, a, b));
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  return ms[ms.size() / 2];
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? std::atof(argv[1]) : 8.0;
  const int rowbytes = 8000;
  const long long nrows = static_cast<long long>(gb * 1e9 / rowbytes);
  double* X;
  double* out;
  CHECK(hipMalloc(&X, nrows * rowbytes + 16384));
  CHECK(hipMemset(X, 0, nrows * rowbytes + 16384));
  CHECK(hipMalloc(&out, sizeof(double) * (1 << 26)));
  const double bytes = static_cast<double>(nrows) * rowbytes;
  // warm the clocks: ~300 ms of streaming
  for (int i = 0; i < 40; ++i) run<0, 2>(X, nrows, rowbytes, 256, out, 1);
  for (int rpw : {64, 256, 768}) {
    const float m0 = run<0, 2>(X, nrows, rowbytes, rpw, out, 15);
    const float m2 = run<2, 2>(X, nrows, rowbytes, rpw, out, 15);
    const float m1 = run<1, 2>(X, nrows, rowbytes, rpw, out, 15);
    const float m0b = run<0, 4>(X, nrows, rowbytes, rpw, out, 15);
    const float m2b = run<2, 4>(X, nrows, rowbytes, rpw, out, 15);
    const float m0c = run<0, 2>(X, nrows, rowbytes, rpw, out, 15);
    std::printf("{\"gb\": %.2f, \"rows_per_wave\": %d, \"default_2infl_TBps\": %.3f, \"nt_2infl_TBps\": %.3f, "
                "\"sc0_2infl_TBps\": %.3f, \"default_4infl_TBps\": %.3f, \"nt_4infl_TBps\": %.3f, \"default_2infl_again_TBps\": %.3f}\n",
                bytes / 1e9, rpw, bytes / m0 / 1e9, bytes / m2 / 1e9, bytes / m1 / 1e9, bytes / m0b / 1e9, bytes / m2b / 1e9,
                bytes / m0c / 1e9);
    std::fflush(stdout);
  }
  CHECK(hipFree(X));
  CHECK(hipFree(out));
  return 0;
}
