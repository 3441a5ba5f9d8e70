// Instruction-rate probes for the f64 path tracer (not shipped): f64/f32 FMA throughput and
// dependent latency, v_rcp_f64 throughput, dependent scalar-load (s_load) latency.
// hipcc --offload-arch=gfx950 -O3 tools_gpu/microbench.hip -o build/microbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

template <int CH>
__global__ void __launch_bounds__(256) fma64(double* out, double a, double b, int iters) {
  double x[CH];
#pragma unroll
  for (int k = 0; k < CH; ++k) x[k] = threadIdx.x * 1e-3 + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int k = 0; k < CH; ++k) x[k] = __builtin_fma(x[k], a, b);
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) s += x[k];
  if (s == 12345.678) out[0] = s;
}

template <int CH>
__global__ void __launch_bounds__(256) fma32(float* out, float a, float b, int iters) {
  float x[CH];
#pragma unroll
  for (int k = 0; k < CH; ++k) x[k] = threadIdx.x * 1e-3f + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int k = 0; k < CH; ++k) x[k] = __builtin_fmaf(x[k], a, b);
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) s += x[k];
  if (s == 12345.678f) out[0] = s;
}

template <int CH>
__global__ void __launch_bounds__(256) rcp64(double* out, int iters) {
  double x[CH];
#pragma unroll
  for (int k = 0; k < CH; ++k) x[k] = 1.0 + threadIdx.x * 1e-3 + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int k = 0; k < CH; ++k) x[k] = __builtin_amdgcn_rcp(x[k]);
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) s += x[k];
  if (s == 12345.678) out[0] = s;
}

// 32-bit integer multiply (v_mul_lo_u32) and xor throughput, 8 independent chains
template <int OP>
__global__ void __launch_bounds__(256) int32op(unsigned* out, unsigned a, int iters) {
  unsigned x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 7u + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[k]) : "v"(a));
        else if (OP == 1) x[k] = (x[k] ^ a) + k;
        else asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[k]) : "v"(a));
      }
  }
  unsigned s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += x[k];
  if (s == 0xdeadbeef) out[0] = s;
}
// f64 compare + select (v_cmp_f64 / v_cndmask_b32 x2) throughput, 8 chains
__global__ void __launch_bounds__(256) cmpsel64(double* out, double a, int iters) {
  double x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 1e-3 + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        double y = x[k];
        asm volatile("" : "+v"(y));
        x[k] = x[k] < a ? y : a;
      }
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += x[k];
  if (s == 12345.678) out[0] = s;
}

// dependent scalar loads: a wave-uniform pointer chase through a small table
__global__ void __launch_bounds__(256) schase(const unsigned* __restrict__ tab, unsigned* out,
                                              int iters) {
  unsigned p = 0;
  for (int i = 0; i < iters; ++i) {
    p = __builtin_amdgcn_readfirstlane(tab[p]);
  }
  if (p == 0xdeadbeef) out[0] = p;
}

static float time_it(void (*launch)(int), int grid) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch(grid);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  launch(grid);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

static double* g_d;
static float* g_f;
static unsigned* g_tab;
static unsigned* g_u;
static const int ITERS = 4096;

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, cus, prop.clockRate);
  CHECK(hipMalloc(&g_d, 64));
  CHECK(hipMalloc(&g_f, 64));
  CHECK(hipMalloc(&g_u, 64));
  const int NT = 4096;
  unsigned h[NT];
  for (int i = 0; i < NT; ++i) h[i] = (i * 2654435761u + 97u) % NT;
  CHECK(hipMalloc(&g_tab, sizeof(h)));
  CHECK(hipMemcpy(g_tab, h, sizeof(h), hipMemcpyHostToDevice));

  // waves per SIMD w: grid = cus * w blocks of 256 threads (4 waves, one per SIMD)
  for (int w : {1, 2, 4, 8}) {
    const int grid = cus * w;
    const double waves = (double)grid * 4;
    const double simds = cus * 4.0;
    auto report = [&](const char* name, float ms, double ops_per_lane) {
      // cycles per wave-instruction per SIMD at the nominal clock
      double wave_instr = waves * ops_per_lane;
      double cyc = ms * 1e-3 * prop.clockRate * 1e3 * simds / wave_instr;
      printf("w/SIMD %d %-22s %8.3f ms  %6.2f cyc/wave-instr/SIMD  %7.2f Tops(lane)/s\n", w, name,
             ms, cyc, wave_instr * 64 / (ms * 1e-3) / 1e12);
    };
    report("fma64 dep (1 chain)", time_it([](int g) { fma64<1><<<g, 256>>>(g_d, 0.999, 1e-3, ITERS); }, grid), ITERS * 8.0);
    report("fma64 4 chains", time_it([](int g) { fma64<4><<<g, 256>>>(g_d, 0.999, 1e-3, ITERS); }, grid), ITERS * 32.0);
    report("fma64 8 chains", time_it([](int g) { fma64<8><<<g, 256>>>(g_d, 0.999, 1e-3, ITERS); }, grid), ITERS * 64.0);
    report("fma32 dep (1 chain)", time_it([](int g) { fma32<1><<<g, 256>>>(g_f, 0.999f, 1e-3f, ITERS); }, grid), ITERS * 8.0);
    report("fma32 8 chains", time_it([](int g) { fma32<8><<<g, 256>>>(g_f, 0.999f, 1e-3f, ITERS); }, grid), ITERS * 64.0);
    report("rcp64 dep (1 chain)", time_it([](int g) { rcp64<1><<<g, 256>>>(g_d, ITERS); }, grid), ITERS * 8.0);
    report("rcp64 8 chains", time_it([](int g) { rcp64<8><<<g, 256>>>(g_d, ITERS); }, grid), ITERS * 64.0);
    report("s_load chase", time_it([](int g) { schase<<<g, 256>>>(g_tab, g_u, ITERS); }, grid), ITERS * 1.0);
    report("mul_lo_u32 8 chains", time_it([](int g) { int32op<0><<<g, 256>>>(g_u, 2654435761u, ITERS); }, grid), ITERS * 64.0);
    report("v_xad_u32 8 chains", time_it([](int g) { int32op<1><<<g, 256>>>(g_u, 2654435761u, ITERS); }, grid), ITERS * 64.0);
    report("mul_u32_u24 8 chains", time_it([](int g) { int32op<2><<<g, 256>>>(g_u, 2654435761u, ITERS); }, grid), ITERS * 64.0);
    report("cmp f64+2 cndmask 8ch", time_it([](int g) { cmpsel64<<<g, 256>>>(g_d, 0.5, ITERS); }, grid), ITERS * 64.0);
  }
  return 0;
}
