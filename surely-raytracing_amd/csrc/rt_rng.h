// rt_rng.h — counter-keyed per-sample RNG of the device path.
//
// The reference draws every random number from rand::thread_rng (ChaCha12, OS-seeded,
// utils.rs:5-15), so it is unseeded and its draw order depends on rayon scheduling. Here each
// pixel-sample owns an independent stream keyed by (seed, global pixel index, sample index):
// pcg2d (Jarzynski & Olano 2020) hashes the key into the state of xoroshiro64* (64 bits of
// state: two VGPRs); draws are then consumed in exactly the reference's call order. Results are
// reproducible and independent of how pixels are distributed over lanes, waves or GPUs. The CPU
// oracle implements the same generator (oracle/rt_oracle.c). Round 5 replaced xoshiro128**
// (removed in round 6): the generator step was 8.2 % of C2 and 17.5 % of C3 by the RT_ABL_RNG2
// ablation (profiles/r05h_abl_rng_c{2,3}.log), and xoroshiro64**'s shorter step and state took
// 0.4 % / 0.95 % off their kernel time (profiles/r05h_x64_c{2,3}.log). Round 6 keyed it with
// pcg2d instead of pcg4d (rng_seed) and took the * scrambler (rng_step).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtd {

struct Rng {
  uint32_t s0, s1;
};
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
// The stream key: pcg2d (Jarzynski & Olano 2020) of (pixel, sample), its two LCG increments keyed
// by the 64-bit seed. Every step is a bijection, so distinct (pixel, sample) pairs of one seed get
// distinct states. The seed words are wave-uniform (scalar ALU); per lane the hash costs six
// v_mul_lo_u32 where round 5's pcg4d of (pixel, sample, seed_lo, seed_hi) cost ten, and the
// camera-ray block that seeds runs in nearly every bounce iteration of a wave.
__device__ __forceinline__ Rng rng_seed(uint32_t seed_lo, uint32_t seed_hi, uint32_t pixel,
                                        uint32_t sample) {
  const uint32_t k0 = (seed_lo ^ 0x85EBCA6Bu) * 0x9E3779B9u + 1013904223u;
  const uint32_t k1 = (seed_hi ^ 0xC2B2AE35u) * 0x9E3779B9u + (k0 ^ 0x27D4EB2Fu);
  uint32_t v0 = pixel * 1664525u + k0, v1 = sample * 1664525u + k1;
  v0 += v1 * 1664525u;
  v1 += v0 * 1664525u;
  v0 ^= v0 >> 16;
  v1 ^= v1 >> 16;
  v0 += v1 * 1664525u;
  v1 += v0 * 1664525u;
  v0 ^= v0 >> 16;
  v1 ^= v1 >> 16;
  if ((v0 | v1) == 0u) v0 = 0x9E3779B9u;  // xoroshiro64*'s state must not be all zero
  return {v0, v1};
}
// xoroshiro64* (Blackman and Vigna): 32-bit outputs from 64 bits of state. The * scrambler (one
// multiply) is the authors' generator for floating-point draws: its weak lowest bits land below
// 2^-24 of a draw (random_double) or are discarded (random_int, a multiply-high). Round 5 used the
// ** scrambler (a rotate and a second multiply on top; profiles/r06g_ab_rngstar_c{2,3,4}.log).
__device__ __forceinline__ uint32_t rng_step(Rng& g) {
  const uint32_t s0 = g.s0;
  uint32_t s1 = g.s1;
  const uint32_t result = s0 * 0x9E3779BBu;
  s1 ^= s0;
  g.s0 = rotl32(s0, 26) ^ s1 ^ (s1 << 9);
  g.s1 = rotl32(s1, 13);
  return result;
}
#ifdef RT_ABL_RNG2
// ablation build (not shipped): every draw's generator step also runs on a copy of the state,
// whose result is discarded (same image); the time delta is the generator's cost
__device__ __forceinline__ uint32_t rng_u32(Rng& g) {
  Rng c = g;
  asm volatile("" : "+v"(c.s0), "+v"(c.s1));
  const uint32_t x = rng_step(c);
  asm volatile("" ::"v"(x), "v"(c.s0), "v"(c.s1));
  return rng_step(g);
}
#else
__device__ __forceinline__ uint32_t rng_u32(Rng& g) { return rng_step(g); }
#endif
// random_double (utils.rs:5-7): 32-bit uniform in [0, 1), exact in f64
__device__ __forceinline__ double rnd(Rng& g) { return (double)rng_u32(g) * 0x1p-32; }
// random_range(-1, 1) (utils.rs:9-11): -1 + 2 * (u * 2^-32) = u * 2^-31 - 1, every step exact
// (u has 32 significant bits, the sum at most 33), so one fma gives the same bits as the
// reference's two operations (the oracle computes them as written)
__device__ __forceinline__ double rnd_pm1(Rng& g) {
  return __builtin_fma((double)rng_u32(g), 0x1p-31, -1.0);
}
// random_int(0, n-1) (utils.rs:13-15): multiply-high
__device__ __forceinline__ uint32_t rnd_index(Rng& g, uint32_t n) { return __umulhi(rng_u32(g), n); }

}  // namespace rtd
