// Common device helpers for the DANSE frame-update engine (gfx950 / CDNA4).
//
// Complex numbers are float2 {re, im}; all arithmetic is fp32 unless a kernel
// is instantiated with double for the solve.  Cross-lane traffic inside a
// lane group of G lanes (G = 16: DPP row broadcast, G = 64: v_readlane into an
// SGPR) never goes through LDS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DANSE_DEV __device__ __forceinline__

struct cf {
  float re, im;
};

DANSE_DEV cf cmk(float r, float i) { return cf{r, i}; }
DANSE_DEV cf operator+(cf a, cf b) { return cf{a.re + b.re, a.im + b.im}; }
DANSE_DEV cf operator-(cf a, cf b) { return cf{a.re - b.re, a.im - b.im}; }
DANSE_DEV cf operator*(cf a, cf b) { return cf{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
DANSE_DEV cf operator*(float s, cf a) { return cf{s * a.re, s * a.im}; }
DANSE_DEV cf conjg(cf a) { return cf{a.re, -a.im}; }
DANSE_DEV float abs2(cf a) { return a.re * a.re + a.im * a.im; }
// a * conj(b)
DANSE_DEV cf mulc(cf a, cf b) { return cf{a.re * b.re + a.im * b.im, a.im * b.re - a.re * b.im}; }
// conj(a) * b
DANSE_DEV cf cmul(cf a, cf b) { return cf{a.re * b.re + a.im * b.im, a.re * b.im - a.im * b.re}; }
// acc += a * b
DANSE_DEV void fma_c(cf& acc, cf a, cf b) {
  acc.re = fmaf(a.re, b.re, fmaf(-a.im, b.im, acc.re));
  acc.im = fmaf(a.re, b.im, fmaf(a.im, b.re, acc.im));
}
// acc -= a * b
DANSE_DEV void fms_c(cf& acc, cf a, cf b) {
  acc.re = fmaf(-a.re, b.re, fmaf(a.im, b.im, acc.re));
  acc.im = fmaf(-a.re, b.im, fmaf(-a.im, b.re, acc.im));
}
// acc -= a * conj(b)
DANSE_DEV void fms_cc(cf& acc, cf a, cf b) {
  acc.re = fmaf(-a.re, b.re, fmaf(-a.im, b.im, acc.re));
  acc.im = fmaf(-a.im, b.re, fmaf(a.re, b.im, acc.im));
}
// The same three operations as two v_pk_fma_f32 each, with the operand
// halves picked and negated by op_sel / neg modifiers (clang materialises
// the swapped and negated pairs with v_mov / v_xor instead: ~1 extra VALU
// op per complex FMA).  Rounding is identical to the scalar forms above
// (same inner / outer fma order per component).
typedef float f2v __attribute__((ext_vector_type(2)));
// acc += a * b
DANSE_DEV void pk_fma_c(cf& acc, cf a, cf b) {
  f2v c = {acc.re, acc.im};
  const f2v x = {a.re, a.im}, y = {b.re, b.im};
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]\n\t"
      "v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]"
      : "+v"(c)
      : "v"(x), "v"(y));
  acc = cf{c.x, c.y};
}
// acc -= a * conj(b)
DANSE_DEV void pk_fms_cc(cf& acc, cf a, cf b) {
  f2v c = {acc.re, acc.im};
  const f2v x = {a.re, a.im}, y = {b.re, b.im};
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]\n\t"
      "v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1] neg_lo:[1,0,0] neg_hi:[1,0,0]"
      : "+v"(c)
      : "v"(x), "v"(y));
  acc = cf{c.x, c.y};
}
// acc += a * conj(b)
DANSE_DEV void pk_fma_cc(cf& acc, cf a, cf b) {
  f2v c = {acc.re, acc.im};
  const f2v x = {a.re, a.im}, y = {b.re, b.im};
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]\n\t"
      "v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]"
      : "+v"(c)
      : "v"(x), "v"(y));
  acc = cf{c.x, c.y};
}
// Generic packed complex multiply-accumulate: acc += (NEG ? -1 : 1) op(a) op(b),
// op = conj where CA / CB.  Inner v_pk_fma_f32: the a.im terms
// (lo: -a.im b.im, hi: a.im b.re, signs folded into neg_lo / neg_hi of
// src0), outer: the a.re terms (lo: a.re b.re, hi: a.re b.im).
#define DANSE_PK_CMAC(N1L, N1H, N2L, N2H)                                                                  \
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[" #N1L ",0,0] neg_hi:[" #N1H \
      ",0,0]\n\tv_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1] neg_lo:[" #N2L ",0,0] neg_hi:[" #N2H ",0,0]" \
      : "+v"(c)                                                                                            \
      : "v"(x), "v"(y))
template <bool CA, bool CB, bool NEG>
DANSE_DEV void cmac(cf& acc, cf a, cf b) {
  constexpr int sA = CA ? -1 : 1, sB = CB ? -1 : 1, s = NEG ? -1 : 1;
  constexpr int code = ((-s * sA * sB) < 0 ? 8 : 0) | ((s * sA) < 0 ? 4 : 0) | (s < 0 ? 2 : 0) | ((s * sB) < 0 ? 1 : 0);
  f2v c = {acc.re, acc.im};
  const f2v x = {a.re, a.im}, y = {b.re, b.im};
  if constexpr (code == 0) DANSE_PK_CMAC(0, 0, 0, 0);
  else if constexpr (code == 1) DANSE_PK_CMAC(0, 0, 0, 1);
  else if constexpr (code == 2) DANSE_PK_CMAC(0, 0, 1, 0);
  else if constexpr (code == 3) DANSE_PK_CMAC(0, 0, 1, 1);
  else if constexpr (code == 4) DANSE_PK_CMAC(0, 1, 0, 0);
  else if constexpr (code == 5) DANSE_PK_CMAC(0, 1, 0, 1);
  else if constexpr (code == 6) DANSE_PK_CMAC(0, 1, 1, 0);
  else if constexpr (code == 7) DANSE_PK_CMAC(0, 1, 1, 1);
  else if constexpr (code == 8) DANSE_PK_CMAC(1, 0, 0, 0);
  else if constexpr (code == 9) DANSE_PK_CMAC(1, 0, 0, 1);
  else if constexpr (code == 10) DANSE_PK_CMAC(1, 0, 1, 0);
  else if constexpr (code == 11) DANSE_PK_CMAC(1, 0, 1, 1);
  else if constexpr (code == 12) DANSE_PK_CMAC(1, 1, 0, 0);
  else if constexpr (code == 13) DANSE_PK_CMAC(1, 1, 0, 1);
  else if constexpr (code == 14) DANSE_PK_CMAC(1, 1, 1, 0);
  else DANSE_PK_CMAC(1, 1, 1, 1);
  acc = cf{c.x, c.y};
}
#undef DANSE_PK_CMAC
DANSE_DEV cf cdiv_real(cf a, float s) {
  float r = 1.0f / s;
  return cf{a.re * r, a.im * r};
}

// Complex double: the noise SCM Rnn and its Cholesky factor (the filter
// update is conditioned by cond(Rnn); see DESIGN.md "Precision").
struct cd {
  double re, im;
};
// Component-wise select.  (A conditional operator on the struct values
// makes clang emit a phi of temporaries' addresses, which keeps the
// operands out of registers: scratch traffic.)
DANSE_DEV cd cdk(cf a) { return cd{(double)a.re, (double)a.im}; }
DANSE_DEV cf cfk(cd a) { return cf{(float)a.re, (float)a.im}; }
DANSE_DEV cd conjg(cd a) { return cd{a.re, -a.im}; }
DANSE_DEV cd operator+(cd a, cd b) { return cd{a.re + b.re, a.im + b.im}; }
DANSE_DEV cd operator-(cd a, cd b) { return cd{a.re - b.re, a.im - b.im}; }
DANSE_DEV cd operator*(double s, cd a) { return cd{s * a.re, s * a.im}; }
// acc += a * b
DANSE_DEV void fma_c(cd& acc, cd a, cd b) {
  acc.re = fma(a.re, b.re, fma(-a.im, b.im, acc.re));
  acc.im = fma(a.re, b.im, fma(a.im, b.re, acc.im));
}
// acc -= a * b
DANSE_DEV void fms_c(cd& acc, cd a, cd b) {
  acc.re = fma(-a.re, b.re, fma(a.im, b.im, acc.re));
  acc.im = fma(-a.re, b.im, fma(-a.im, b.re, acc.im));
}
// acc += a * conj(b)
DANSE_DEV void fma_cc(cd& acc, cd a, cd b) {
  acc.re = fma(a.re, b.re, fma(a.im, b.im, acc.re));
  acc.im = fma(a.im, b.re, fma(-a.re, b.im, acc.im));
}
// acc -= a * conj(b)
DANSE_DEV void fms_cc(cd& acc, cd a, cd b) {
  acc.re = fma(-a.re, b.re, fma(-a.im, b.im, acc.re));
  acc.im = fma(-a.im, b.re, fma(a.re, b.im, acc.im));
}

DANSE_DEV cf csel(bool c, cf a, cf b) { return cf{c ? a.re : b.re, c ? a.im : b.im}; }
DANSE_DEV cd csel(bool c, cd a, cd b) { return cd{c ? a.re : b.re, c ? a.im : b.im}; }

DANSE_DEV int lane_id() { return __lane_id(); }

// Register values a straight run of loads just produced, pinned here: the
// loads issue back to back and are waited for once.  Without it the compiler
// sinks each load into the branch (or next to the store) that uses it, and an
// unrolled 16-element loop becomes 16 serial memory round trips -- the z
// chain of bcast_kernel and the observation loads of the lane kernels spent
// most of their time that way.
DANSE_DEV void hold1(float& x) { asm volatile("" : "+v"(x)); }
DANSE_DEV void hold1(int& x) { asm volatile("" : "+v"(x)); }
DANSE_DEV void hold1(double& x) { asm volatile("" : "+v"(x)); }
DANSE_DEV void hold1(cf& x) { asm volatile("" : "+v"(x.re), "+v"(x.im)); }
DANSE_DEV void hold1(cd& x) { asm volatile("" : "+v"(x.re), "+v"(x.im)); }
template <typename T, int n>
DANSE_DEV void hold(T (&x)[n]) {
#pragma unroll
  for (int i = 0; i < n; ++i) hold1(x[i]);
}

// ---------------------------------------------------------------------------
// Lane-group broadcast: value of lane `SRC` of my group of G lanes.
//   G == 64 : v_readlane_b32 (wave-uniform SGPR result)
//   G == 16 : DPP row_newbcast (gfx90a+ "row share"), one VALU op, no LDS
//   G == 4  : DPP quad_perm
//   G == 32 : ds_bpermute
// ---------------------------------------------------------------------------
template <int G, int SRC>
DANSE_DEV float gbcast(float x) {
  static_assert(SRC >= 0 && SRC < G, "source lane out of group");
  if constexpr (G == 64) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), SRC));
  } else if constexpr (G == 4) {
    constexpr int qp = SRC | (SRC << 2) | (SRC << 4) | (SRC << 6);   // DPP quad_perm
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), qp, 0xF, 0xF, true));
  } else if constexpr (G == 16) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x150 + SRC, 0xF, 0xF, true));
  } else {
    int base = (lane_id() & ~(G - 1)) + SRC;
    return __int_as_float(__builtin_amdgcn_ds_bpermute(base << 2, __float_as_int(x)));
  }
}

template <int G, int SRC>
DANSE_DEV cf gbcast(cf x) {
  return cf{gbcast<G, SRC>(x.re), gbcast<G, SRC>(x.im)};
}

// Runtime source lane (wave-uniform for G == 64, group-uniform otherwise).
template <int G>
DANSE_DEV float gbcast_rt(float x, int src) {
  if constexpr (G == 64) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), src));
  } else {
    int base = (lane_id() & ~(G - 1)) + src;
    return __int_as_float(__builtin_amdgcn_ds_bpermute(base << 2, __float_as_int(x)));
  }
}
template <int G>
DANSE_DEV cf gbcast_rt(cf x, int src) {
  return cf{gbcast_rt<G>(x.re, src), gbcast_rt<G>(x.im, src)};
}

// Butterfly exchange inside a DPP row (16 lanes) without LDS:
//   xor 1, xor 2 : quad_perm [1,0,3,2] / [2,3,0,1]
//   half swap    : row_half_mirror (lane i <-> 7 - i, quads 0/1 swap once the
//                  values are quad-uniform)
//   row swap     : row_mirror (lane i <-> 15 - i)
template <int CTRL>
DANSE_DEV float dpp_x(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, true));
}
template <int G, typename Op>
DANSE_DEV float greduce(float x, Op op) {
  static_assert(G == 4 || G == 16 || G == 32 || G == 64, "group size");
  x = op(x, dpp_x<0xB1>(x));
  x = op(x, dpp_x<0x4E>(x));
  if constexpr (G >= 16) {
    x = op(x, dpp_x<0x141>(x));
    x = op(x, dpp_x<0x140>(x));
  }
  if constexpr (G == 32) {
    x = op(x, __shfl_xor(x, 16, 32));
  } else if constexpr (G == 64) {
    const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 0));
    const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 16));
    const float c = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 32));
    const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 48));
    x = op(op(a, b), op(c, d));
  }
  return x;
}

// Sum over the G lanes of my group (result in every lane of the group).
template <int G>
DANSE_DEV float gsum(float x) {
  return greduce<G>(x, [](float a, float b) { return a + b; });
}
template <int G>
DANSE_DEV cf gsum(cf x) {
  return cf{gsum<G>(x.re), gsum<G>(x.im)};
}
template <int G>
DANSE_DEV float gmax(float x) {
  return greduce<G>(x, [](float a, float b) { return fmaxf(a, b); });
}
template <int G>
DANSE_DEV float gmin(float x) {
  return greduce<G>(x, [](float a, float b) { return fminf(a, b); });
}
// Hardware transcendental approximations (1 ulp; no IEEE divide/sqrt
// expansion, no denormal rescaling).
DANSE_DEV float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
DANSE_DEV float frsq(float x) { return __builtin_amdgcn_rsqf(x); }
DANSE_DEV float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
// Group ballot: bit i set if lane i of my group has pred.
template <int G>
DANSE_DEV uint64_t gballot(bool pred) {
  uint64_t b = __ballot(pred);
  if constexpr (G == 64) {
    return b;
  } else {
    const int sh = lane_id() & ~(G - 1);
    return (b >> sh) & ((1ull << G) - 1ull);
  }
}
