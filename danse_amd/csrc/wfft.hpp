// One-WAVEFRONT 1024-point complex FFT (four-step, 1024 = 16 x 64), used by
// the WOLA analysis / synthesis of the broadcast kernel.  A wave owns its FFT:
// no workgroup barrier, so the waves of a workgroup run independent FFTs
// (one per microphone frame, estimate, ...) side by side.
//
//   in : lane l holds x[l + 64 j], j = 0..15              (registers)
//   A  : 16-point DFT over j, twiddle W1024^(l k1)        (registers)
//   T  : transpose through LDS (16 x 68-complex pitch: conflict-free writes
//        and 2-dwords-per-bank reads)
//   B  : lane l = 4 k1 + a: 16-point DFT over b of T[k1][4 b + a],
//        twiddle W64^(a c)                                 (registers)
//   C  : 4-point DFT over a across the lane quad (two DPP radix-2 stages)
//   out: lane l = 4 k1 + a holds X[k1 + 16 c + 256 e], c = 0..15,
//        e = 2 (a & 1) + (a >> 1)
// X[k] = sum_n x[n] exp(-2 pi i k n / 1024).
#pragma once
#include "common.hpp"

namespace danse {
namespace wfft {

constexpr int kPitch = 68;                 // complex elements per LDS row
constexpr int kLdsElems = 16 * kPitch;     // per wave

DANSE_DEV void dft4(cf& x0, cf& x1, cf& x2, cf& x3) {
  const cf a0 = x0 + x2, a1 = x0 - x2, a2 = x1 + x3, d13 = x1 - x3;
  const cf a3 = cf{d13.im, -d13.re};   // -i (x1 - x3)
  x0 = a0 + a2;
  x1 = a1 + a3;
  x2 = a0 - a2;
  x3 = a1 - a3;
}

// W16^m = exp(-2 pi i m / 16), m = 0..15 (compile-time m after unrolling)
DANSE_DEV cf w16(int m) {
  constexpr float c1 = 0.92387953251128674f, s1 = 0.38268343236508978f, h = 0.70710678118654752f;
  switch (m & 15) {
    case 0: return cf{1.0f, 0.0f};
    case 1: return cf{c1, -s1};
    case 2: return cf{h, -h};
    case 3: return cf{s1, -c1};
    case 4: return cf{0.0f, -1.0f};
    case 5: return cf{-s1, -c1};
    case 6: return cf{-h, -h};
    case 7: return cf{-c1, -s1};
    case 8: return cf{-1.0f, 0.0f};
    case 9: return cf{-c1, s1};
    case 10: return cf{-h, h};
    case 11: return cf{-s1, c1};
    case 12: return cf{0.0f, 1.0f};
    case 13: return cf{s1, c1};
    case 14: return cf{h, h};
    default: return cf{c1, s1};
  }
}

// In-register 16-point DFT, natural order in and out (n = 4p + q,
// k = r + 4s: radix-4 over p, twiddle W16^(q r), radix-4 over q).
DANSE_DEV void dft16(cf (&x)[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) dft4(x[q], x[q + 4], x[q + 8], x[q + 12]);   // A[q][r] at x[4r + q]
#pragma unroll
  for (int q = 1; q < 4; ++q) {
#pragma unroll
    for (int r = 1; r < 4; ++r) x[4 * r + q] = x[4 * r + q] * w16(q * r);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) dft4(x[4 * r], x[4 * r + 1], x[4 * r + 2], x[4 * r + 3]);   // X[r + 4s] at x[4r + s]
  cf y[16];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int s = 0; s < 4; ++s) y[r + 4 * s] = x[4 * r + s];
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = y[i];
}

template <int CTRL>
DANSE_DEV cf dpp(cf v) {
  return cf{__int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v.re), CTRL, 0xF, 0xF, true)),
            __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v.im), CTRL, 0xF, 0xF, true))};
}

DANSE_DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Twiddle table of the wave FFT (kTwElems complex, built in double on the
// host at engine creation): [k1][l] = W1024^(l k1) (16 x 64, so every load of
// a wave is 512 contiguous bytes), then [a][c] = W64^(a c) (4 x 16).
constexpr int kTwElems = 16 * 64 + 4 * 16;

// Forward FFT of the wave's 1024 points (layout above), the twiddles from
// TW: tw1(k1) = W1024^(l k1), k1 = 1..15, and tw2(c) = W64^(a c), c = 1..15.
template <typename TW>
DANSE_DEV void fft1024_tw(cf (&v)[16], cf* lds, const TW& tw) {
  const int l = __lane_id();
  // A: DFT over j, twiddle W1024^(l k1)
  dft16(v);
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) v[k1] = v[k1] * tw.tw1(k1);
  wave_sync();   // the previous FFT's reads of lds are done
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) lds[k1 * kPitch + l] = v[k1];
  wave_sync();
  // B: lane (k1, a) = (l >> 2, l & 3): DFT over b of T[k1][4b + a]
  const int k1 = l >> 2, a = l & 3;
#pragma unroll
  for (int b = 0; b < 16; ++b) v[b] = lds[k1 * kPitch + 4 * b + a];
  dft16(v);
#pragma unroll
  for (int c = 1; c < 16; ++c) v[c] = v[c] * tw.tw2(c);
  // C: 4-point DFT over a across the quad.  Stage 1 pairs a, a ^ 2
  // (a1 = a >> 1 becomes e0, twiddle W4^(a0 e0)), stage 2 pairs a, a ^ 1
  // (a0 becomes e1).
  const bool hi1 = (a & 2) != 0, hi0 = (a & 1) != 0;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const cf p = dpp<0x4E>(v[c]);   // quad_perm [2,3,0,1]: lane a ^ 2
    cf t = hi1 ? p - v[c] : v[c] + p;
    if (hi1 && hi0) t = cf{t.im, -t.re};   // x (-i)
    const cf q = dpp<0xB1>(t);            // quad_perm [1,0,3,2]: lane a ^ 1
    v[c] = hi0 ? q - t : t + q;
  }
}

// twiddles read from the kTwElems table in memory
struct TwMem {
  const cf* __restrict__ tw;
  DANSE_DEV cf tw1(int k1) const { return tw[k1 * 64 + __lane_id()]; }
  DANSE_DEV cf tw2(int c) const { return tw[16 * 64 + (__lane_id() & 3) * 16 + c]; }
};
// twiddles held in registers (a persistent wave that transforms every round)
struct TwReg {
  cf t1[16], t2[16];
  DANSE_DEV void load(const cf* __restrict__ tw) {
#pragma unroll
    for (int i = 1; i < 16; ++i) {
      t1[i] = tw[i * 64 + __lane_id()];
      t2[i] = tw[16 * 64 + (__lane_id() & 3) * 16 + i];
    }
  }
  DANSE_DEV cf tw1(int k1) const { return t1[k1]; }
  DANSE_DEV cf tw2(int c) const { return t2[c]; }
};

DANSE_DEV void fft1024(cf (&v)[16], cf* lds, const cf* __restrict__ tw) { fft1024_tw(v, lds, TwMem{tw}); }

// Frequency index of output element c on this lane.
DANSE_DEV int out_index(int c) {
  const int l = __lane_id();
  const int k1 = l >> 2, a = l & 3;
  const int e = ((a & 1) << 1) | (a >> 1);
  return k1 + 16 * c + 256 * e;
}

}  // namespace wfft
}  // namespace danse
