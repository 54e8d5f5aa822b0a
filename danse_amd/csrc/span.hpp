// Pre-solve prefix fast-forward.  Until the first round in which any item
// solves (config N2: 181 of 310 rounds, B: 57), a round's update is the SCM
// recursion (d_classes.py:2048-2267) plus the tail (filter carry, external
// filters, d-hat).  The recursion does not feed back into the broadcasts, so
// the engine defers it: every prefix round copies its update-frame spectra
// and fused spectra into per-round histories and runs only the tail
// (UpdateArgs.noRec), and before the first solving round span_rec_kernel
// runs the whole prefix's recursion per bin, each SCM entry loaded and
// stored once instead of once per round (the recursion-only rounds were
// HBM-bound at ~5 TB/s).  Same arithmetic, entry by entry, as the
// recursion-only kernels (kernels_lane.hpp RO, kernels_2d.hpp SM = 1).
#pragma once
#include "kernels.hpp"

namespace danse {

struct SpanArgs {
  int S, K, MT, F, P, nFN;
  const uint8_t* flags;     // [R][S][kMaxFam][K]
  const FamNode* fn;        // every family-node of the engine (packed 1 or 2)
  const int* chanList;
  const cf* yHist;          // [P][S][MT][F] update-frame spectra of the prefix rounds
  const cf* zHist;          // [P][K][S][F] fused spectra of the prefix rounds
  cf* Ryy;
  cd* Rnn;
  long long scmStride;
  const double* beta;       // [S][K]
};

constexpr int kSpanChunk = 16;    // rounds staged in LDS at once

// a prefix round's two history copies in one launch (complex64 entries):
// the update-frame spectra and the fused spectra
__global__ void __launch_bounds__(256) ff_copy_kernel(cf* __restrict__ dy, const cf* __restrict__ sy, size_t ny,
                                                      cf* __restrict__ dz, const cf* __restrict__ sz, size_t nz) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < ny + nz; i += stride) {
    if (i < ny) dy[i] = sy[i];
    else dz[i - ny] = sz[i - ny];
  }
}

// one THREADS-thread workgroup per (scene, family-node, bin); thread t holds
// the lower entries e = t + THREADS j (j < PER) of both SCMs for the whole
// prefix; YW >= D (the staged observation rows)
template <int THREADS, int PER, int YW>
__global__ void __launch_bounds__(THREADS) span_rec_kernel(const SpanArgs a) {
  __shared__ cf ys[kSpanChunk][YW];
  __shared__ uint8_t ops[kSpanChunk];
  const int F = a.F, tid = threadIdx.x;
  const int f = blockIdx.x % F;
  const int fni = (blockIdx.x / F) % a.nFN;
  const int s = blockIdx.x / (F * a.nFN);
  const FamNode d = a.fn[fni];
  const int D = d.D, NT = D * (D + 1) / 2;
  const double beta = a.beta[s * a.K + d.k];
  const long long base = (long long)s * a.scmStride + d.scmOff;
  auto at = [&](int e) -> long long { return d.packed == 1 ? base + (long long)e * F + f : base + (long long)f * NT + e; };
  int ei[PER], ej[PER];
  cf ry[PER];
  cd rn[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int e = tid + THREADS * j;
    const int ec = e < NT ? e : 0;
    // packed lower triangle: e = i (i + 1) / 2 + c
    int i = (int)((sqrtf(8.0f * ec + 1.0f) - 1.0f) * 0.5f);
    while (i * (i + 1) / 2 > ec) --i;
    while ((i + 1) * (i + 2) / 2 <= ec) ++i;
    ei[j] = i;
    ej[j] = ec - i * (i + 1) / 2;
    ry[j] = a.Ryy[at(ec)];
    rn[j] = a.Rnn[at(ec)];
  }
  const float byf = (float)beta;
  const float cyAvgF = (float)((1.0 - beta) / D), cySetF = (float)(1.0 / D);
  const double cyAvg = (1.0 - beta) / D, cySet = 1.0 / D;
  for (int r0 = 0; r0 < a.P; r0 += kSpanChunk) {
    __syncthreads();
    for (int x = tid; x < kSpanChunk * D; x += THREADS) {
      const int rr = r0 + x / D, i = x % D;
      cf v = cf{0.0f, 0.0f};
      if (rr < a.P) {
        const int c = a.chanList[d.chanOff + i];
        v = (c < a.MT) ? a.yHist[(((long long)rr * a.S + s) * a.MT + c) * F + f]
                       : a.zHist[((((long long)rr * a.K + (c - a.MT)) * a.S + s)) * F + f];
      }
      ys[x / D][i] = v;
    }
    if (tid < kSpanChunk) {
      const int rr = r0 + tid;
      ops[tid] = rr < a.P ? (a.flags[(((long long)rr * a.S + s) * kMaxFam + d.fam) * a.K + d.k] & 15) : 0;
    }
    __syncthreads();
    const int n = min(kSpanChunk, a.P - r0);
    for (int k = 0; k < n; ++k) {
      const int opY = ops[k] & 3, opN = (ops[k] >> 2) & 3;   // (workgroup-uniform)
      if (opY) {
        const float cy = (opY == DANSE_OP_SET) ? cySetF : cyAvgF;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
          const int i = ei[j], c = ej[j];
          const cf yy = cy * mulc(ys[k][i], ys[k][c]);
          cf x = (opY == DANSE_OP_SET) ? yy : byf * ry[j] + yy;
          if (i == c) x.im = 0.0f;
          ry[j] = x;
        }
      }
      if (opN) {
        const double cy = (opN == DANSE_OP_SET) ? cySet : cyAvg;
        const double cx = (opN == DANSE_OP_SET) ? 0.0 : beta;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
          const int i = ei[j], c = ej[j];
          cd yy = cd{0.0, 0.0};
          fma_cc(yy, cdk(ys[k][i]), cdk(ys[k][c]));
          cd x = cx * rn[j];
          x.re = fma(cy, yy.re, x.re);
          x.im = (i == c) ? 0.0 : fma(cy, yy.im, x.im);
          rn[j] = x;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int e = tid + THREADS * j;
    if (e < NT) {
      a.Ryy[at(e)] = ry[j];
      a.Rnn[at(e)] = rn[j];
    }
  }
}

// the instantiation for a size class: 64 threads per bin up to DMAX 20, 256
// above, PER entries per thread
inline void launch_span_class(int DMAX, const SpanArgs& a, unsigned blocks, hipStream_t st) {
  const int nt = DMAX * (DMAX + 1) / 2;
#define DANSE_SPAN(T, P, Y) hipLaunchKernelGGL((span_rec_kernel<T, P, Y>), dim3(blocks), dim3(T), 0, st, a)
  if (DMAX <= 12) DANSE_SPAN(64, 2, 16);
  else if (DMAX <= 16) DANSE_SPAN(64, 3, 16);
  else if (DMAX <= 20) DANSE_SPAN(64, 4, 32);
  else if (nt <= 512) DANSE_SPAN(256, 2, 64);
  else if (nt <= 768) DANSE_SPAN(256, 3, 64);
  else if (nt <= 1024) DANSE_SPAN(256, 4, 64);
  else if (nt <= 1280) DANSE_SPAN(256, 5, 64);
  else if (nt <= 1792) DANSE_SPAN(256, 7, 64);
  else DANSE_SPAN(256, 9, 64);
#undef DANSE_SPAN
}

}  // namespace danse
