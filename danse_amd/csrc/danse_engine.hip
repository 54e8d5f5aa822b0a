// Host side of the C-ABI (include/danse_mi355x.h): engine state, launch
// sequencing, hipGraph capture, and the fine-grained operators.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/danse_mi355x.h"
#include "bcast.hpp"
#include "fill.hpp"
#include "wide_api.hpp"
#include "classes.hpp"
#include "gate.hpp"
#include "cohdrift.hpp"
#include "tzconv.hpp"
#include "resident.hpp"
#include "resident_api.hpp"
#include "cond.hpp"
#include "wide_online.hpp"
#include "span.hpp"

using namespace danse;

namespace {

constexpr int kF = 513;

struct Class {
  int G, DMAX;
  std::vector<FamNode> host;
  std::vector<int> ids;
  FamNode* dev = nullptr;
  int* devIds = nullptr;
  // split solves (lane classes D 9..12, UpdateArgs.splitSolve): per round the
  // items that solve, [R][S * nFN] (the first solveCount[r] of a row used)
  bool split = false;
  int* dSolveItems = nullptr;
  std::vector<int> solveCount;
  // per round: does any item of the class solve (else the recursion-only
  // kernel variant runs)
  std::vector<uint8_t> anySolve;  // solves on the cached factor and C (kernels_2dc.hpp): per round the
  // items for update_kernel_2dc, [R][S * nFN] (the first creCount[r] of a row
  // used), and the fallback list / per-round counters
  bool lean = false;
  bool leanNoise = false;   // (every node's beta > 0: li_rank1_2d)
  int* dCreItems = nullptr;
  int* dCnItems = nullptr;
  std::vector<int> creCount, cnCount;
  int* dFbList = nullptr;
  int* dFbCount = nullptr;
  // lane classes (G = 1), GEVD: the factor records in wave order
  // (UpdateArgs.liLane, [block][entry][64])
  cf* liLane = nullptr;
};

template <typename T>
hipError_t dalloc(T** p, size_t n) {
  if (n == 0) n = 1;
  return hipMalloc((void**)p, n * sizeof(T));
}

}  // namespace

struct danse_engine {
  int dev = 0;
  std::string err;
  int S, K, MT, N, Ns, F, T, R, k0, k1;
  int gevd, rank, ref, families, keepHistory;
  float alphaExt;
  std::vector<int> M, base, extMode;
  std::vector<FamNode> fns;   // all family-nodes (owned nodes)
  std::vector<int> chanList;
  std::vector<Class> classes;
  long long scmStride = 0, wStride = 0, wExtStride = 0, tgtStride = 0;
  std::vector<long long> wExtNodeOff;
  // device
  int *dM = nullptr, *dBase = nullptr, *dBcEnd = nullptr, *dUpEnd = nullptr, *dChan = nullptr;
  uint8_t* dFlags = nullptr;
  uint8_t* dZLag = nullptr;
  double* dZPhase = nullptr;
  double* dBeta = nullptr;
  float *dBetaExt = nullptr, *dhA = nullptr, *dhS = nullptr, *dNorm = nullptr;
  cf* dTw = nullptr;
  long long* dWExtNodeOff = nullptr;
  const float* y = nullptr;
  cd* Rnn = nullptr;   // complex double (DESIGN.md "Precision"); same element offsets as Ryy
  cf *Yspec = nullptr, *Zspec = nullptr, *Ryy = nullptr, *wHist = nullptr, *wExtHist = nullptr,
     *wExtTarget = nullptr, *dhat = nullptr;
  float *zPrev = nullptr, *zStream = nullptr, *d = nullptr;
  int* diag = nullptr;
  hipGraphExec_t graphExec = nullptr;
  int graphR0 = -1, graphR1 = -1;
  void* graphStream = nullptr;
  bool ownZspec = true;
  int foreign = 0;   // BcastArgs.foreign
  bool noRO = false;     // DANSE_NO_RO: never the recursion-only update variants (A/B timing)
  int bcastAblate = 0;   // DANSE_BCAST_ABLATE (diagnostics only; results are wrong when set)
  // initial-state copies for danse_engine_reset
  std::vector<long long> initW0Off, initScmOff, extSrcOff, tgtOff;
  cf *dW0 = nullptr, *dExt0 = nullptr, *dTgt0 = nullptr;
  cd* dScm0 = nullptr;
  cf* liCache = nullptr;     // GEVD factor cache of the lane classes (kernels.hpp li_reusable)
  // speculative gate schedule (danse_engine_set_gate): candidates sorted by
  // round, gateOff[r] .. gateOff[r + 1] checked between bcast(r) and update(r)
  GateCand* dGateCand = nullptr;
  int* dGateVerdict = nullptr;
  std::vector<int> gateOff;
  std::vector<int> gateDmax;   // per round: largest candidate D (LDS size)
  cd* gateWork = nullptr;      // gate_wide_kernel workspace (candidates above kGateMaxD)
  long long gateWorkItems = 0; // (cand, bin) workgroups per chunk
  int nGate = 0;
  // CohDrift (cohdrift.hpp)
  int cohDrift = 0, cdLd = 0, cdStart = 0, cdEvery = 1, cdComp = 0, cdNIter = 0;
  int cdOpen = 0;
  double* cdFlagWin = nullptr;   // open loop: [R][K][K] flag windows (danse_cfg.cdFlagWin)
  double cdAlpha = 0.0, cdAlphaEps = 0.0;
  cd *cdRing = nullptr, *cdAvg = nullptr;
  double *cdPhase = nullptr, *cdEst = nullptr, *cdRes = nullptr;
  long long liStride = 0;
  cf* vCache = nullptr;      // lane-grid GEVD classes: eigenvector of C per bin (warm start)
  long long vStride = 0;
  cd* l64Cache = nullptr;    // lane-grid GEVD classes: float64 factor record per bin (rank-one updates)
  long long l64Stride = 0;
  cf* cCache = nullptr;      // 8 x 8 grid GEVD classes: C = Li Ryy Li^H per bin (UpdateArgs.cCache)
  long long cStride = 0;
  int* lzStats = nullptr;    // [R][2] warm Lanczos solves accepted / sent back (danse_engine_lanczos_stats)
  // the online centralised family above 64 channels (wide_online.hpp)
  std::vector<int> wideIds;          // family-node indices
  std::vector<uint8_t> wideSolve;    // [R][wideIds]: some scene solves
  int* dWideIds = nullptr;
  cd* wideWork = nullptr;
  long long wideChunk = 0;
  int scmPerBin = 0;   // dScm0 holds [F][D][D] per family-node (else [D][D])
  FamNode* dFnAll = nullptr;
  long long *dInitW0Off = nullptr, *dInitScmOff = nullptr, *dExtSrcOff = nullptr, *dTgtOff = nullptr;
  // fewSamples broadcasts (cfg.fsTab): T(z) IRs [S][K][Mmax][2N-1], schedule
  int zLen = 0, Mmax = 0;
  std::vector<int> fsTab;          // host copy [R][K][DANSE_FS_FIELDS] (ZEND per consuming round)
  int* dFsTab = nullptr;
  // the fewSamples device steps (danse_cfg.fsSteps): chunk rows [nEv][K][FIELDS],
  // steps [n][DANSE_FS_STEP_FIELDS], first step of each round [R + 1]
  std::vector<int> fsEv, fsSteps, fsRoundStep;
  int* dFsEv = nullptr;
  float* rawStream = nullptr;      // [S][MT][zLen] (cfg.rawStreams)
  float* zChunk = nullptr;         // node-sharded DXCP: [K][S][Ns] exchange buffer (borrowed)
  float *wIR = nullptr, *dSn = nullptr;
  // desSigProcessingType 'conv' (danse_cfg.desSigConv): per-family-node T(z)
  // IRs of the new filter's first M_k columns [S][nFN][Mmax][2N - 1] and the
  // window cross-correlation table of dist_fct_approx(w, win_s, win_s, Ns)
  int desConv = 0;
  float *convIR = nullptr, *dSnConv = nullptr;
  // DXCP-PhaT SRO estimation in the loop (cfg.dxcp, an extension: the
  // reference's integration raises, quirk Q12): one estimator per (scene,
  // receiver, sender), fed every kDxEvery rounds
  int dxcpOn = 0;
  danse_dxcp* dx = nullptr;
  float* dxFrames = nullptr;     // [P][2][2048]
  double *dxOut = nullptr, *dxEst = nullptr;   // [P][2], [S][K][K] current estimate (relative SRO)
  // record of every feed's gathered frames and estimator outputs
  // (danse_engine_dxcp_record): [nFeeds][P][2][2048] f32, [nFeeds][P][2] f64
  float* dxRecFrames = nullptr;
  double* dxRecOut = nullptr;
  int dxRecFeeds = 0;
  // centralised / SSBC raw frames under asynchronous clocks (cfg.cEnd)
  int* dCEnd = nullptr;
  cf* Cspec = nullptr;
  int* dChanNode = nullptr;
  double* dCPhase = nullptr;
  // resident engine (danse_engine_run_resident, resident.hpp)
  std::vector<std::pair<int, GateCand>> gateHost;   // the installed gate schedule (round, candidate)
  cf *resYB = nullptr, *resYU = nullptr, *resZall = nullptr, *resZhat = nullptr, *resRyyG = nullptr;
  cd* resRnnG = nullptr;
  unsigned *resUFlag = nullptr, *resZFlag = nullptr;
  int *resGateRound = nullptr, *resDanseFni = nullptr, *resErr = nullptr, *resFams = nullptr;
  float* resFrames = nullptr;
  int* resChanNode = nullptr;        // [MT] node of each channel
  unsigned long long* resTrace = nullptr;   // DANSE_RESIDENT_TRACE / DANSE_UPDATE_TRACE diagnostics
  size_t resTraceBytes = 0;
  int updTraceRound = -1;   // DANSE_UPDATE_TRACE=r: stamp build's per-wave marks of round r's update launch
  int resNFam = 0;
  // condition numbers of Ryy (cond.hpp), every condEvery-th iteration
  int condEvery = 0;
  // pre-solve prefix fast-forward (span.hpp): rounds [0, ffP) run the tail
  // only, their recursion in one span_rec_kernel before round ffP; ffPraw
  // from the flag table (build_split_lists), ffAlloc the histories' rounds
  int ffP = 0, ffPraw = 0, ffAlloc = 0;
  // a launch error inside a launch helper that has no return path (the wide
  // filter chunks): sticky until the next entry point reports it
  hipError_t launchErr = hipSuccess;
  bool ffOk = false;
  cf *yHist = nullptr, *zHist = nullptr;
  double* condHist = nullptr;   // [S][nFN][R][F]
};

static thread_local std::string g_lastErr;

#define HIPCHK(expr)                                                                  \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) {                                                           \
      std::string m = std::string(#expr) + ": " + hipGetErrorString(_e);              \
      if (eng) eng->err = m;                                                          \
      g_lastErr = m;                                                                  \
      return -2;                                                                      \
    }                                                                                 \
  } while (0)

static int fail(danse_engine* eng, const std::string& m) {
  if (eng) eng->err = m;
  g_lastErr = m;
  return -1;
}

// the sticky launch error of a helper (launch_wide), reported once
static int take_launch_err(danse_engine* eng) {
  if (!eng || eng->launchErr == hipSuccess) return 0;
  const hipError_t e = eng->launchErr;
  eng->launchErr = hipSuccess;
  return fail(eng, std::string("wide filter launch: ") + hipGetErrorString(e));
}

// The size class a filter dimension runs on: class_dmax, except that
// DANSE_D20_ON_G8=1 moves D 17..20 from the 4 x 4 grid class 20 (four bins per
// wave) to the 8 x 8 grid class 24 (one bin per wave), which carries the
// float64 factor records and the lean cached-C solves (A/B)
static int eng_class_dmax(int D) {
  const char* e = std::getenv("DANSE_D20_ON_G8");
  const bool g8 = e && std::atoi(e) != 0;
  return (g8 && D > 16 && D <= 20) ? 24 : class_dmax(D);
}
static void pick_class(int D, int& G, int& DMAX) {
  DMAX = eng_class_dmax(D);
  G = class_group(DMAX);
}
// (G = 1: lane kernels on packed SCMs; 16: lane groups; 64: one bin per wave)

// Re-initialise filters (slot 0 of the histories) and SCMs of every
// (scene, family-node): one block row per (scene, family-node).
__global__ void reset_fam_kernel(const FamNode* fns, int nFN, const long long* w0Off, const long long* scmOff,
                                 const cf* w0, const cd* scm0, cf* wHist, long long wStride, cf* Ryy, cd* Rnn,
                                 long long scmStride, int F, int perBin) {
  const int s = blockIdx.y / nFN;
  const int i = blockIdx.y % nFN;
  const FamNode fn = fns[i];
  const int D = fn.D;
  const long long T = (long long)D * (D + 1) / 2;
  const long long nS = fn.packed ? F * T : (long long)F * D * D;
  const long long nW = (long long)F * D;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < nS; e += (long long)gridDim.x * blockDim.x) {
    long long src;
    if (fn.packed) {
      // packed entry t = i (i + 1) / 2 + j of bin fb -> full slice element (i, j)
      const int t = (int)(fn.packed == 1 ? e / F : e % T);
      const long long fb = fn.packed == 1 ? e % F : e / T;
      int r = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
      while (r * (r + 1) / 2 > t) --r;
      while ((r + 1) * (r + 2) / 2 <= t) ++r;
      src = (long long)r * D + (t - r * (r + 1) / 2);
      if (perBin) src += fb * D * D;
    } else {
      src = perBin ? e : e % ((long long)D * D);
    }
    const cd v = scm0[scmOff[i] + src];
    Ryy[s * scmStride + fn.scmOff + e] = cfk(v);
    Rnn[s * scmStride + fn.scmOff + e] = v;
    if (fn.D > kMaxDMax) Rnn[s * scmStride + fn.scmOff + nS + e] = v;   // (the wide fns' float64 Ryy)
    if (e < nW) wHist[s * wStride + fn.wOff + e] = w0[w0Off[i] + e];
  }
}

__global__ void reset_ext_kernel(const int* M, int k0, int k1, const long long* srcOff, const long long* dstOff,
                                 const long long* tgtOff, const cf* ext0, const cf* tgt0, cf* wExtHist,
                                 long long wExtStride, cf* tgt, long long tgtStride, int F) {
  const int nOwn = k1 - k0;
  const int s = blockIdx.y / nOwn;
  const int k = k0 + blockIdx.y % nOwn;
  const long long n = (long long)F * M[k];
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    wExtHist[s * wExtStride + dstOff[k] + e] = ext0[srcOff[k] + e];
    tgt[s * tgtStride + tgtOff[k] + e] = tgt0[srcOff[k] + e];
  }
}

// ---- fewSamples broadcasts (tzconv.hpp) -------------
struct FsArgs {
  int S, K, MT, T, N, F, r, k0, k1, Mmax, ref, keepHistory, zLen;
  const int* M;
  const int* base;
  const int* fsTab;          // [R][K][DANSE_FS_FIELDS]
  const float* y;            // [S][MT][T]
  const cf* wExtHist;
  const long long* wExtNodeOff;
  long long wExtStride;
  const cf* tw;              // wave-FFT twiddles
  const float* sn;           // window correlation / (N Ns), [2N-1]
  float* wIR;                // [S][K][Mmax][2N-1]
  float* zStream;            // [S][K][zLen]
  float* rawStream;          // [S][MT][zLen] raw-sample streams of the centralised buffers, or null
  int foreign;               // (BcastArgs.foreign) the chunk grid covers every node; the blocks of the
                             // nodes not owned append the raw samples only
};

DANSE_DEV const int* fs_entry(const FsArgs& a, int k) { return a.fsTab + ((long long)a.r * a.K + k) * DANSE_FS_FIELDS; }

// T(z) IR refresh (dist_fct_approx of wExt[i], d_classes.py:1093-1106): one
// wave per (scene, owned node, sensor); nodes without a refresh this round
// exit as whole waves.
__global__ void __launch_bounds__(256) fs_ir_kernel(const FsArgs a) {
  __shared__ cf lds[4][wfft::kLdsElems];
  const int wv = threadIdx.x >> 6;
  const int nOwn = a.k1 - a.k0;
  const int item = blockIdx.x * 4 + wv;
  if (item >= a.S * nOwn * a.Mmax) return;
  const int m = item % a.Mmax;
  const int s = item / (nOwn * a.Mmax);
  const int k = a.k0 + (item / a.Mmax) % nOwn;
  const int Mk = a.M[k];
  const int src = fs_entry(a, k)[DANSE_FS_IRSRC];
  if (m >= Mk || src < 0) return;
  const int slot = a.keepHistory ? src : (src & 1);
  const cf* w = a.wExtHist + (long long)s * a.wExtStride + a.wExtNodeOff[k] + (long long)slot * a.F * Mk + m;
  float* o = a.wIR + (((long long)s * a.K + k) * a.Mmax + m) * tzc::kA;
  tzc::ir_wave(lds[wv], a.tw, a.sn, [&](int f) { return w[(long long)f * Mk]; }, [&](int t, float v) { o[t] = v; });
}

// The currL samples node k broadcasts (danse_compression_few_samples,
// d_base.py:1871-1938) appended to its stream at POS (fill_buffers,
// d_classes.py:1185-1224): one workgroup per (scene, owned node).
__global__ void __launch_bounds__(tzc::kThr) fs_chunk_kernel(const FsArgs a) {
  __shared__ tzc::ConvLds sm;
  const int nGrid = a.foreign ? a.K : a.k1 - a.k0;
  const int s = blockIdx.x / nGrid;
  const int k = (a.foreign ? 0 : a.k0) + blockIdx.x % nGrid;
  const bool owned = k >= a.k0 && k < a.k1;
  const int* e = fs_entry(a, k);
  const int L = e[DANSE_FS_LEN];
  if (L <= 0) return;   // uniform per workgroup
  const int end = e[DANSE_FS_BCEND];
  const int Mk = a.M[k];
  const float* y = a.y + ((long long)s * a.MT + a.base[k]) * a.T;
  const float* ir = a.wIR + ((long long)s * a.K + k) * a.Mmax * tzc::kA;
  float* z = a.zStream + ((long long)s * a.K + k) * a.zLen + e[DANSE_FS_POS];
  const int T = a.T, N = a.N;
  if (owned)   // (block-uniform)
  tzc::conv_block(
      sm, Mk, L,
      [&](int q, int m) {   // local_chunk_for_broadcast: y[end - N + q] (clamped read), zero before sample 0
        return y[(long long)m * T + min(max(end - N + q, 0), T - 1)];
      },
      [&](int q, int) { return end - N + q >= 0 && end - N + q < T; },
      [&](int i, int m) { return ir[(long long)m * tzc::kA + i]; }, [&](int i, float v) { z[i] = v; });
  if (a.rawStream) {
    // the raw samples the centralised buffers receive with the chunk
    // (pre_fill_buffers_centralised + fill_buffers_centr, d_classes.py:
    // 1162-1250: the last currL samples of the broadcast frame, zero before 0)
    const int pos = e[DANSE_FS_POS];
    for (int m = 0; m < Mk; ++m) {
      float* o = a.rawStream + ((long long)s * a.MT + a.base[k] + m) * a.zLen + pos;
      for (int i = threadIdx.x; i < L; i += blockDim.x) {
        const int idx = end - L + i;
        o[i] = (idx >= 0 && idx < T) ? y[(long long)m * T + idx] : 0.0f;
      }
    }
  }
}

// Initial IR: a Dirac at tap N on the reference sensor (d_classes.py:660-663).
__global__ void fs_ir_init_kernel(float* wIR, int K, int Mmax, int ref, int N) {
  const int sk = blockIdx.x;
  if (threadIdx.x == 0) wIR[((long long)sk * Mmax + ref) * tzc::kA + N] = 1.0f;
}

// ---- DXCP-PhaT in the loop (extension; SURVEY §8e "DXCP per node pair after
// the z all-gather").  Every kDxEvery = 2048 / Ns rounds each receiver k
// feeds its estimator of sender q with the 2048 newest samples of its
// local reference sensor (ending at the update frame end upEnd[r][k]) and of
// q's fused-signal stream as k has received it ((r + 1 - zLag) Ns samples):
// consecutive, non-overlapping DXCP-PhaT frames (sro_estimation.py:208-227).
// The estimate of q's sampling rate relative to k's, eps_kq = -SRO ppm 1e-6
// (DXCP-PhaT reports the second channel's sampling-period excess), replaces
// the Oracle value of update_sro_estimates (d_classes.py:2364-2621): the
// sender's phase accumulator loses eps Ns after every round's update.
constexpr int kDxFrame = 2048;
__global__ void __launch_bounds__(256) dxcp_gather_kernel(const UpdateArgs a, const int* upEnd, const float* y,
                                                          const float* zStream, int zLen, int T, int Ns,
                                                          const int* base, int ref, int k0, int nOwn,
                                                          float* frames) {
  const int K = a.K, r = a.r;
  const int qi = blockIdx.x % (K - 1);
  const int k = k0 + (int)((blockIdx.x / (K - 1)) % nOwn);
  const int s = blockIdx.x / ((K - 1) * nOwn);
  const int q = qi < k ? qi : qi + 1;
  const int e0 = upEnd[r * K + k];
  const int lag = a.zLag ? a.zLag[((long long)r * K + k) * K + q] : 0;
  const long long zEnd = (long long)(r + 1 - lag) * Ns;
  const float* yl = y + ((long long)s * a.MT + base[k] + ref) * T;
  const float* zs = zStream + ((long long)s * K + q) * zLen;
  float* f = frames + (long long)blockIdx.x * 2 * kDxFrame;
  for (int n = threadIdx.x; n < kDxFrame; n += blockDim.x) {
    const long long iy = (long long)e0 - kDxFrame + n, iz = zEnd - kDxFrame + n;
    f[n] = (iy >= 0 && iy < T) ? yl[iy] : 0.0f;
    f[kDxFrame + n] = (iz >= 0 && iz < zLen) ? zs[iz] : 0.0f;
  }
}

// after round r's update: new DXCP estimates on feeding rounds, then the
// phase accumulation and the SROsEstimates / SROsResiduals rows of round r
__global__ void dxcp_round_kernel(int S, int K, int k0, int nOwn, int r, int R, int fed, int compensate, double Ns,
                                  const double* dxOut, double* est, double* phase, double* estHist,
                                  double* resHist) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= S * nOwn * (K - 1)) return;
  const int qi = p % (K - 1);
  const int k = k0 + (p / (K - 1)) % nOwn;
  const int s = p / ((K - 1) * nOwn);
  const int q = qi < k ? qi : qi + 1;
  double* e = est + ((long long)s * K + k) * K + q;
  if (fed) *e = -dxOut[2 * p] * 1e-6;
  const double v = *e;
  const long long o = (((long long)s * K + k) * R + r) * (K - 1) + qi;
  resHist[o] = v;
  estHist[o] = compensate ? v : 0.0;
  if (compensate) phase[((long long)s * K + k) * K + q] -= v * Ns;
}

int danse_engine_reset(danse_engine* eng, void* stream) {
  if (!eng) return fail(eng, "null engine");
  HIPCHK(hipSetDevice(eng->dev));
  hipStream_t st = (hipStream_t)stream;
  const int S = eng->S, K = eng->K, F = eng->F, R = eng->R;
  HIPCHK(fill_async(eng->zPrev, 0, (size_t)S * K * eng->N * sizeof(float), st));
  if (eng->dxcpOn) {
    HIPCHK(fill_async(eng->dxEst, 0, (size_t)S * K * K * sizeof(double), st));
    if (danse_dxcp_reset(eng->dx, st) != 0) return fail(eng, std::string("DXCP estimator: ") + danse_dxcp_last_error(eng->dx));
  }
  if (eng->cohDrift || eng->dxcpOn) {
    HIPCHK(fill_async(eng->cdPhase, 0, (size_t)S * K * K * sizeof(double), st));
    HIPCHK(fill_async(eng->cdEst, 0, (size_t)S * K * (K - 1) * R * sizeof(double), st));
    HIPCHK(fill_async(eng->cdRes, 0, (size_t)S * K * (K - 1) * R * sizeof(double), st));
  }
  HIPCHK(fill_async(eng->Zspec, 0, (size_t)2 * K * S * F * sizeof(cf), st));
  if (eng->Cspec) HIPCHK(fill_async(eng->Cspec, 0, (size_t)2 * S * eng->MT * F * sizeof(cf), st));
  HIPCHK(fill_async(eng->zStream, 0, (size_t)S * K * eng->zLen * sizeof(float), st));
  if (eng->rawStream) HIPCHK(fill_async(eng->rawStream, 0, (size_t)S * eng->MT * eng->zLen * sizeof(float), st));
  if (eng->wIR) {
    HIPCHK(fill_async(eng->wIR, 0, (size_t)S * K * eng->Mmax * tzc::kA * sizeof(float), st));
    hipLaunchKernelGGL(fs_ir_init_kernel, dim3(S * K), dim3(64), 0, st, eng->wIR, K, eng->Mmax, eng->ref, eng->N);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(fill_async(eng->dhat, 0, (size_t)kMaxFam * S * K * R * F * sizeof(cf), st));
  HIPCHK(fill_async(eng->d, 0, (size_t)kMaxFam * S * K * eng->T * sizeof(float), st));
  HIPCHK(fill_async(eng->diag, 0, (size_t)S * K * kMaxFam * sizeof(int), st));
  if (eng->vCache) HIPCHK(fill_async(eng->vCache, 0, (size_t)S * eng->vStride * sizeof(cf), st));
  if (eng->lzStats) HIPCHK(fill_async(eng->lzStats, 0, (size_t)2 * eng->R * kLzSlots * sizeof(int), st));
  for (auto& cl : eng->classes)
    if (cl.dFbCount) HIPCHK(fill_async(cl.dFbCount, 0, ((size_t)eng->R + 1) * sizeof(int), st));
  const int nFN = (int)eng->fns.size();
  hipLaunchKernelGGL(reset_fam_kernel, dim3(64, S * nFN), dim3(256), 0, st, eng->dFnAll, nFN, eng->dInitW0Off,
                     eng->dInitScmOff, eng->dW0, eng->dScm0, eng->wHist, eng->wStride, eng->Ryy, eng->Rnn,
                     eng->scmStride, F, eng->scmPerBin);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(reset_ext_kernel, dim3(8, S * (eng->k1 - eng->k0)), dim3(256), 0, st, eng->dM, eng->k0, eng->k1,
                     eng->dExtSrcOff, eng->dWExtNodeOff, eng->dTgtOff, eng->dExt0, eng->dTgt0, eng->wExtHist,
                     eng->wExtStride, eng->wExtTarget, eng->tgtStride, F);
  HIPCHK(hipGetLastError());
  if (st == nullptr) HIPCHK(hipDeviceSynchronize());
  return 0;
}

const char* danse_last_error(const danse_engine* eng) {
  if (eng && !eng->err.empty()) return eng->err.c_str();
  return g_lastErr.c_str();
}

// The split classes' per-round lists of solving (scene, family-node) items.
// per round and wide family-node: does some scene solve (the wide filter
// launch is skipped otherwise)
static void build_wide_lists(danse_engine* eng, const uint8_t* flags) {
  const int nW = (int)eng->wideIds.size(), R = eng->R, S = eng->S, K = eng->K;
  eng->wideSolve.assign((size_t)R * nW, 0);
  for (int r = 0; r < R; ++r)
    for (int w = 0; w < nW; ++w) {
      const FamNode& fn = eng->fns[eng->wideIds[w]];
      for (int s = 0; s < S; ++s) {
        const uint8_t fl = flags[(((size_t)r * S + s) * kMaxFam + fn.fam) * K + fn.k];
        if ((fl & DANSE_FLAG_SOLVE) && !(fl & DANSE_FLAG_PREGIVEN)) eng->wideSolve[(size_t)r * nW + w] = 1;
      }
    }
}

static int build_split_lists(danse_engine* eng, const uint8_t* flags) {
  const int S = eng->S, K = eng->K, R = eng->R;
  {
    // the pre-solve prefix: the rounds before the first solve of any item
    // and before the first round at which the frame counters allow a start
    // (the reference gate's check reads the SCMs there: ny > D and nn > D,
    // the counts of the rounds whose Ryy / Rnn op is not KEEP)
    int P = R;
    const int nf = (int)eng->fns.size();
    for (int t = 0; t < S * nf; ++t) {
      const FamNode& d = eng->fns[t % nf];
      int ny = 0, nn = 0;
      for (int r = 0; r < P; ++r) {
        const uint8_t fl = flags[(((size_t)r * S + t / nf) * kMaxFam + d.fam) * K + d.k];
        ny += (fl & 3) != 0;
        nn += ((fl >> 2) & 3) != 0;
        if (((fl & DANSE_FLAG_SOLVE) && !(fl & DANSE_FLAG_PREGIVEN)) || (ny > d.D && nn > d.D)) {
          P = r;
          break;
        }
      }
    }
    eng->ffPraw = (P < R && P >= 8) ? P : 0;
    eng->ffP = eng->ffOk ? std::min(eng->ffPraw, eng->ffAlloc) : 0;
  }
  for (auto& cl : eng->classes) {
    const int nn = (int)cl.host.size();
    cl.anySolve.assign(R, 0);
    for (int r = 0; r < R; ++r)
      for (int t = 0; t < S * nn && !cl.anySolve[r]; ++t) {
        const FamNode& d = cl.host[t % nn];
        const uint8_t fl = flags[(((size_t)r * S + t / nn) * kMaxFam + d.fam) * K + d.k];
        if ((fl & DANSE_FLAG_SOLVE) && !(fl & DANSE_FLAG_PREGIVEN)) cl.anySolve[r] = 1;
      }
    if (cl.lean) {
      // (the host mirror of the kernels' reuse tests: kernels.hpp li_reusable
      // and c_reusable -- a solve, no Rnn update this round, and a solve of
      // this item since the last SCM update within kLiScan rounds)
      auto flag = [&](int r, int t) {
        const FamNode& d = cl.host[t % nn];
        return flags[(((size_t)r * S + t / nn) * kMaxFam + d.fam) * K + d.k];
      };
      std::vector<int> items((size_t)R * S * nn, 0), nitems((size_t)R * S * nn, 0);
      cl.creCount.assign(R, 0);
      cl.cnCount.assign(R, 0);
      for (int r = 0; r < R; ++r)
        for (int t = 0; t < S * nn; ++t) {
          const uint8_t fl = flag(r, t);
          const int opY = fl & 3, opN = (fl >> 2) & 3;
          if (!(fl & DANSE_FLAG_SOLVE) || (fl & DANSE_FLAG_PREGIVEN)) continue;
          const bool vad = opN == DANSE_OP_KEEP;
          const bool noise = cl.leanNoise && opN == DANSE_OP_AVG && opY == DANSE_OP_KEEP;
          if ((!vad && !noise) || cl.host[t % nn].cOff < 0 || r % kCRefresh == 0) continue;
          bool ok = false;
          for (int rr = r - 1; rr >= 0 && rr >= r - kLiScan; --rr) {
            const uint8_t f2 = flag(rr, t);
            if ((f2 & DANSE_FLAG_SOLVE) && !(f2 & DANSE_FLAG_PREGIVEN)) { ok = true; break; }
            if (f2 & 15) break;
          }
          if (!ok) continue;
          if (vad) items[(size_t)r * S * nn + cl.creCount[r]++] = t;
          else nitems[(size_t)r * S * nn + cl.cnCount[r]++] = t;
        }
      if (!cl.dCreItems) HIPCHK(dalloc(&cl.dCreItems, items.size()));
      if (!cl.dCnItems) HIPCHK(dalloc(&cl.dCnItems, nitems.size()));
      HIPCHK(hipMemcpy(cl.dCreItems, items.data(), items.size() * sizeof(int), hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(cl.dCnItems, nitems.data(), nitems.size() * sizeof(int), hipMemcpyHostToDevice));
    }
    if (!cl.split) continue;
    const int n = (int)cl.host.size();
    std::vector<int> items((size_t)R * S * n, 0);
    cl.solveCount.assign(R, 0);
    for (int r = 0; r < R; ++r)
      for (int t = 0; t < S * n; ++t) {
        const FamNode& d = cl.host[t % n];
        const uint8_t fl = flags[(((size_t)r * S + t / n) * kMaxFam + d.fam) * K + d.k];
        if ((fl & DANSE_FLAG_SOLVE) && !(fl & DANSE_FLAG_PREGIVEN)) items[(size_t)r * S * n + cl.solveCount[r]++] = t;
      }
    if (!cl.dSolveItems) HIPCHK(dalloc(&cl.dSolveItems, items.size()));
    HIPCHK(hipMemcpy(cl.dSolveItems, items.data(), items.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  return 0;
}

int danse_engine_create(const danse_cfg* c, int device, danse_engine** out) {
  danse_engine* eng = nullptr;
  if (!c || !out) return fail(nullptr, "null argument");
  if (c->N != 1024) return fail(nullptr, "only DFTsize 1024 is supported by the HIP FFT");
  if (c->K < 2 || c->S < 1 || c->R < 1) return fail(nullptr, "bad sizes");
  if (c->k0 < 0 || c->k1 > c->K || c->k0 >= c->k1) return fail(nullptr, "bad owned node range");
  if (c->rank < 1 || c->rank > kRMax) return fail(nullptr, "GEVD rank out of range [1, 4]");
  eng = new danse_engine();
  eng->dev = device;
  if (const char* ab = std::getenv("DANSE_BCAST_ABLATE")) eng->bcastAblate = std::atoi(ab);
  eng->noRO = std::getenv("DANSE_NO_RO") != nullptr;
  HIPCHK(hipSetDevice(device));
  eng->S = c->S; eng->K = c->K; eng->N = c->N; eng->Ns = c->Ns; eng->F = c->N / 2 + 1; eng->T = c->T;
  eng->R = c->R; eng->k0 = c->k0; eng->k1 = c->k1; eng->gevd = c->gevd; eng->rank = c->rank; eng->ref = c->ref;
  eng->families = c->families | 1; eng->keepHistory = c->keepHistory; eng->alphaExt = c->alphaExt;
  eng->foreign = (c->k0 != 0 || c->k1 != c->K) &&
                 (eng->families & ((1 << DANSE_FAM_CENTR) | (1 << DANSE_FAM_SSBC))) ? 1 : 0;
  const int K = c->K, S = c->S, F = eng->F, R = c->R;
  eng->M.assign(c->M, c->M + K);
  for (int k = 0; k < K; ++k) eng->Mmax = std::max(eng->Mmax, eng->M[k]);
  eng->zLen = c->fsTab ? c->zStreamLen : R * c->Ns;
  if (eng->zLen < 1) return fail(eng, "zStreamLen must be positive with fsTab");
  if (c->fsTab) {
    eng->fsTab.assign(c->fsTab, c->fsTab + (size_t)R * K * DANSE_FS_FIELDS);
    for (int r = 0; r < R; ++r)
      for (int k = 0; k < K; ++k) {
        const int* e = &eng->fsTab[((size_t)r * K + k) * DANSE_FS_FIELDS];
        if (e[DANSE_FS_ZEND] < 0 || e[DANSE_FS_ZEND] > eng->zLen) return fail(eng, "fewSamples z frame end outside the stream");
      }
    if (K > 31) return fail(eng, "fewSamples steps: at most 31 nodes (node masks)");
    const int all = (1 << K) - 1;
    if (c->fsSteps) {
      // (a round is at least BCAST + UPDATE; chunk steps only where a stream
      // needs one -- the per-step validation below checks every round)
      if (!c->fsEv || c->nFsSteps < 2 * R || c->nFsEv < 0) return fail(eng, "fewSamples steps: too few steps or no chunk rows");
      eng->fsEv.assign(c->fsEv, c->fsEv + (size_t)c->nFsEv * K * DANSE_FS_FIELDS);
      eng->fsSteps.assign(c->fsSteps, c->fsSteps + (size_t)c->nFsSteps * DANSE_FS_STEP_FIELDS);
    } else {   // one CHUNK (fsTab row r), BCAST, UPDATE per round
      eng->fsEv = eng->fsTab;
      for (int r = 0; r < R; ++r) {
        const int st[3][4] = {{DANSE_FS_STEP_CHUNK, r, all, r}, {DANSE_FS_STEP_BCAST, r, all, -1},
                              {DANSE_FS_STEP_UPDATE, r, all, -1}};
        for (auto& x : st) eng->fsSteps.insert(eng->fsSteps.end(), x, x + 4);
      }
    }
    // validate: rounds contiguous and in order, one BCAST per round and before
    // its updates, every node updated once per round, a chunk's IR source
    // written before it (and still in the two-slot ring without history)
    const int nSt = (int)(eng->fsSteps.size() / DANSE_FS_STEP_FIELDS);
    const int nEv = (int)(eng->fsEv.size() / ((size_t)K * DANSE_FS_FIELDS));
    std::vector<int> done(K, 0);
    eng->fsRoundStep.assign(R + 1, nSt);
    int cur = -1, upd = 0, bc = 0;
    for (int i = 0; i < nSt; ++i) {
      const int* x = &eng->fsSteps[(size_t)i * DANSE_FS_STEP_FIELDS];
      const int ty = x[0], r = x[1], mask = x[2], row = x[3];
      if (r != cur) {
        if (r != cur + 1 || r >= R || (cur >= 0 && (upd != all || !bc))) return fail(eng, "fewSamples steps out of round order");
        cur = r; upd = 0; bc = 0;
        eng->fsRoundStep[r] = i;
      }
      if (mask & ~all) return fail(eng, "fewSamples step mask names a missing node");
      if (ty == DANSE_FS_STEP_CHUNK) {
        if (row < 0 || row >= nEv) return fail(eng, "fewSamples chunk row out of range");
        for (int k = 0; k < K; ++k) {
          const int* e = &eng->fsEv[((size_t)row * K + k) * DANSE_FS_FIELDS];
          if (e[DANSE_FS_LEN] < 0 || e[DANSE_FS_LEN] > c->N) return fail(eng, "fewSamples chunk length outside [0, N]");
          if (e[DANSE_FS_POS] < 0 || e[DANSE_FS_POS] + e[DANSE_FS_LEN] > eng->zLen)
            return fail(eng, "fewSamples chunk outside the stream");
          if (e[DANSE_FS_IRSRC] > done[k] || e[DANSE_FS_IRSRC] < -1)
            return fail(eng, "IR refresh from a wExt iteration not yet written");
          if (!c->keepHistory && e[DANSE_FS_IRSRC] >= 0 && e[DANSE_FS_IRSRC] < done[k] - 1)
            return fail(eng, "IR refresh from an old wExt iteration needs keepHistory");
        }
      } else if (ty == DANSE_FS_STEP_BCAST) {
        if (bc || upd) return fail(eng, "fewSamples BCAST step after an update of its round");
        bc = 1;
      } else if (ty == DANSE_FS_STEP_ZAN) {
        if (!bc) return fail(eng, "fewSamples z analysis before its round's BCAST");
      } else if (ty == DANSE_FS_STEP_UPDATE) {
        if (!bc || (upd & mask)) return fail(eng, "fewSamples update step out of order");
        upd |= mask;
        for (int k = 0; k < K; ++k)
          if ((mask >> k) & 1) done[k] = r + 1;
      } else {
        return fail(eng, "unknown fewSamples step type");
      }
    }
    if (cur != R - 1 || upd != all || !bc) return fail(eng, "fewSamples steps do not cover every round");
    eng->fsRoundStep[R] = nSt;
  }
  eng->extMode.assign(c->extMode, c->extMode + K);
  eng->base.resize(K);
  int mt = 0;
  for (int k = 0; k < K; ++k) { eng->base[k] = mt; mt += eng->M[k]; }
  eng->MT = mt;
  if (c->ref < 0) return fail(eng, "bad reference sensor");
  for (int k = 0; k < K; ++k)
    if (c->ref >= eng->M[k]) return fail(eng, "referenceSensor must be < M_k for every node");

  // ---- family-node table (owned nodes), channel lists; with cEnd the other
  // nodes' channels of the centralised / SSBC vectors are raw-frame codes
  // (MT + K + channel, kernels.hpp load_y)
  long long scmOff = 0, wOff = 0, liOff = 0, vOff = 0, l64Off = 0, cOff = 0;
  // warm-started rank-1 Lanczos on the lane-grid classes (DANSE_NO_WARM=1: off)
  const bool warm = c->gevd && c->rank == 1 && !std::getenv("DANSE_NO_WARM");
  const int rawBase = mt + K;
  const long long histW = c->keepHistory ? (long long)R + 1 : 2;
  for (int fam = 0; fam < kMaxFam; ++fam) {
    if (!((eng->families >> fam) & 1)) continue;
    for (int k = c->k0; k < c->k1; ++k) {
      FamNode fn{};
      fn.fam = fam; fn.k = k; fn.M = eng->M[k]; fn.extMode = (fam == DANSE_FAM_DANSE) ? eng->extMode[k] : -1;
      fn.chanOff = (int)eng->chanList.size();
      if (fam == DANSE_FAM_DANSE || fam == DANSE_FAM_SSBC) {
        for (int m = 0; m < eng->M[k]; ++m) eng->chanList.push_back(eng->base[k] + m);
        for (int q = 0; q < K; ++q)
          if (q != k)
            eng->chanList.push_back(fam == DANSE_FAM_DANSE ? mt + q : (c->cEnd ? rawBase : 0) + eng->base[q]);
        fn.D = eng->M[k] + K - 1;
        fn.ref = c->ref;
      } else if (fam == DANSE_FAM_LOCAL) {
        for (int m = 0; m < eng->M[k]; ++m) eng->chanList.push_back(eng->base[k] + m);
        fn.D = eng->M[k];
        fn.ref = c->ref;
      } else {
        for (int q = 0; q < K; ++q)
          for (int m = 0; m < eng->M[q]; ++m)
            eng->chanList.push_back((q != k && c->cEnd ? rawBase : 0) + eng->base[q] + m);
        fn.D = mt;
        fn.ref = eng->base[k] + c->ref;
      }
      if (fn.D > kMaxDMax) {
        // (only the centralised family reaches past 64 channels: the wide
        // classes of wide_online.hpp, synchronous wholeChunk runs, the gate's
        // matrix in LDS up to kGateMaxD)
        if (fam != DANSE_FAM_CENTR || fn.D > wide::kMaxD)
          return fail(eng, "filter dimension > 64 outside the centralised family, or a centralised family above 256 channels");
        if (c->cEnd || c->fsTab || c->cPhase)
          return fail(eng, "centralised family above 64 channels: synchronous wholeChunk runs only");
      }
      if (c->gevd && c->rank > fn.D) return fail(eng, "GEVD rank larger than a filter dimension");
      fn.scmOff = scmOff;
      // smallDGrid: GEVD of D <= 12 on the 4 x 4 grid class 16; the grid and
      // row classes keep bin-major triangles (FamNode.packed 2)
      const bool gridSmall = c->smallDGrid && c->gevd && fn.D <= kLaneMaxD;
      fn.packed = (class_packed(fn.D) && !gridSmall) ? 1 : 2;
      // (the wide fns keep Ryy in float64 past their Rnn: kernels.hpp wide_fn)
      scmOff += (long long)F * fn.D * (fn.D + 1) / 2 * (fn.D > kMaxDMax ? 2 : 1);
      fn.wOff = wOff;
      wOff += histW * F * fn.D;
      fn.liOff = liOff;
      const bool wideFn = fn.D > kMaxDMax;
      // (a split class's grid solves keep their own per-bin record in the region)
      if (wideFn) {
        // (no factor caches: the wide solve factors every time)
      } else if (c->gevd && fn.packed == 1)
        liOff += (long long)F * std::max<long long>(fn.D * (fn.D + 1) / 2 + fn.D,
                                                    class_split(eng_class_dmax(fn.D)) ? class_split_li_record() : 0);
      else if (c->gevd && gridSmall) liOff += (long long)F * class_li_record(16);
      else if (c->gevd && class_grid(eng_class_dmax(fn.D)) > 0) liOff += (long long)F * class_li_record(eng_class_dmax(fn.D));
      fn.vOff = -1;
      fn.l64Off = -1;
      // float64 factor records (li_rank1_2d) of the one-bin-per-wave grid
      // classes (DMAX 24-48; at G = 4, DMAX <= 20, the O(D^3) factor is short
      // and the update measured slower: C 360 -> 372 us, N2 263 -> 255 us)
      if (!wideFn && c->gevd && fn.packed == 2 && !gridSmall && class_grid(eng_class_dmax(fn.D)) > 0 &&
          eng_class_dmax(fn.D) >= 24 && !std::getenv("DANSE_NO_R1")) {
        const int DMr = eng_class_dmax(fn.D);
        fn.l64Off = l64Off;
        l64Off += (long long)F * (DMr * (DMr + 1) / 2 + DMr);
      }
      // (grid classes of 20 and more: solver2d.hpp gevd2d_filter)
      if (!wideFn && warm && fn.packed == 2 && !gridSmall && class_grid(eng_class_dmax(fn.D)) > 0 && eng_class_dmax(fn.D) >= 20) {
        fn.vOff = vOff;
        vOff += (long long)F * eng_class_dmax(fn.D);
      }
      // C = Li Ryy Li^H per bin (kernels_2d.hpp): the 8 x 8 grid classes with
      // the warm start and the float64 factor record (DANSE_NO_CCACHE=1: off)
      fn.cOff = -1;
      if (fn.vOff >= 0 && fn.l64Off >= 0 && class_grid(eng_class_dmax(fn.D)) == 8 && !std::getenv("DANSE_NO_CCACHE")) {
        const long long nb = eng_class_dmax(fn.D) / 8;
        fn.cOff = cOff;
        cOff += (long long)F * nb * (nb + 1) / 2 * 64;   // (kernels_2d.hpp c_record)
      } else if (fn.vOff >= 0 && class_grid(eng_class_dmax(fn.D)) == 4 && !std::getenv("DANSE_NO_CCACHE")) {
        // the 4 x 4 grid class (four bins per wave): one record per bin group
        // of four (kernels_2d.hpp c4_ptr), used inside update_kernel_2d
        const long long nb = eng_class_dmax(fn.D) / 4;
        fn.cOff = cOff;
        cOff += (long long)((F + 3) / 4) * nb * (nb + 1) / 2 * 64;
      }
      eng->fns.push_back(fn);
    }
  }
  eng->scmStride = scmOff;
  eng->wStride = wOff;
  eng->liStride = liOff;
  eng->vStride = vOff;
  eng->l64Stride = l64Off;
  eng->cStride = cOff;
  eng->wExtNodeOff.assign(K, 0);
  long long eo = 0, to = 0;
  for (int k = 0; k < K; ++k) {
    eng->wExtNodeOff[k] = eo;
    eo += histW * F * eng->M[k];
  }
  eng->wExtStride = eo;
  std::vector<long long> tgtOff(K);
  for (int k = 0; k < K; ++k) { tgtOff[k] = to; to += (long long)F * eng->M[k]; }
  eng->tgtStride = to;
  for (auto& fn : eng->fns) {
    if (fn.fam == DANSE_FAM_DANSE) { fn.wExtOff = eng->wExtNodeOff[fn.k]; fn.tgtOff = tgtOff[fn.k]; }
  }
  for (size_t i = 0; i < eng->fns.size(); ++i) {
    if (eng->fns[i].D > kMaxDMax) {
      eng->wideIds.push_back((int)i);
      continue;
    }
    int G, DM;
    pick_class(eng->fns[i].D, G, DM);
    if (eng->fns[i].packed == 2 && DM <= kLaneMaxD) {   // smallDGrid (above)
      G = class_group(16);
      DM = 16;
    }
    Class* cl = nullptr;
    for (auto& x : eng->classes)
      if (x.G == G && x.DMAX == DM) cl = &x;
    if (!cl) { eng->classes.push_back(Class{G, DM, {}, {}, nullptr, nullptr}); cl = &eng->classes.back(); }
    cl->host.push_back(eng->fns[i]);
    cl->ids.push_back((int)i);
  }

  // ---- device allocations
  HIPCHK(dalloc(&eng->dM, K));
  HIPCHK(dalloc(&eng->dBase, K));
  HIPCHK(dalloc(&eng->dBcEnd, (size_t)R * K));
  HIPCHK(dalloc(&eng->dUpEnd, (size_t)R * K));
  HIPCHK(dalloc(&eng->dChan, eng->chanList.size()));
  HIPCHK(dalloc(&eng->dFlags, (size_t)R * S * kMaxFam * K));
  HIPCHK(dalloc(&eng->dBeta, (size_t)S * K));
  HIPCHK(dalloc(&eng->dBetaExt, (size_t)S * K));
  HIPCHK(dalloc(&eng->dhA, (size_t)c->N));
  HIPCHK(dalloc(&eng->dhS, (size_t)c->N));
  HIPCHK(dalloc(&eng->dNorm, (size_t)c->Ns));
  HIPCHK(dalloc(&eng->dTw, (size_t)c->N + wfft::kTwElems));
  HIPCHK(dalloc(&eng->dWExtNodeOff, (size_t)K));
  HIPCHK(hipMemcpy(eng->dM, eng->M.data(), K * sizeof(int), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->dBase, eng->base.data(), K * sizeof(int), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->dBcEnd, c->bcEnd, (size_t)R * K * sizeof(int), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->dUpEnd, c->upEnd, (size_t)R * K * sizeof(int), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->dChan, eng->chanList.data(), eng->chanList.size() * sizeof(int), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->dFlags, c->flags, (size_t)R * S * kMaxFam * K, hipMemcpyHostToDevice));
  if (c->zLag) {
    HIPCHK(dalloc(&eng->dZLag, (size_t)R * K * K));
    HIPCHK(hipMemcpy(eng->dZLag, c->zLag, (size_t)R * K * K, hipMemcpyHostToDevice));
  }
  if (c->zPhase) {
    HIPCHK(dalloc(&eng->dZPhase, (size_t)R * K * K));
    HIPCHK(hipMemcpy(eng->dZPhase, c->zPhase, (size_t)R * K * K * sizeof(double), hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemcpy(eng->dBeta, c->beta, (size_t)S * K * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->dBetaExt, c->betaExt, (size_t)S * K * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->dhA, c->winAnalysis, c->N * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->dhS, c->winSynthesis, c->N * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->dWExtNodeOff, eng->wExtNodeOff.data(), K * sizeof(long long), hipMemcpyHostToDevice));
  {
    // OLA normalisation h^2[n] + h^2[n + Ns] (d_base.py:1843-1852), in double then rounded
    std::vector<float> nv(c->Ns);
    const int nOv = c->N / c->Ns;
    std::vector<double> acc(c->N + c->Ns, 0.0);
    for (int ii = 0; ii < nOv; ++ii)
      for (int n = 0; n < c->N; ++n) acc[ii * c->Ns + n] += (double)c->winAnalysis[n] * c->winAnalysis[n];
    for (int n = 0; n < c->Ns; ++n) nv[n] = (float)acc[c->Ns + n];
    HIPCHK(hipMemcpy(eng->dNorm, nv.data(), c->Ns * sizeof(float), hipMemcpyHostToDevice));
    std::vector<cf> tw(c->N);
    for (int m = 0; m < c->N; ++m) {
      const double ang = -2.0 * M_PI * (double)m / (double)c->N;
      tw[m] = cf{(float)std::cos(ang), (float)std::sin(ang)};
    }
    // [0, N): exp(-2 pi i m / N) (workgroup FFT); then the wave-FFT table
    for (int k1 = 0; k1 < 16; ++k1)
      for (int l = 0; l < 64; ++l) {
        const double ang = -2.0 * M_PI * (double)(l * k1) / 1024.0;
        tw.push_back(cf{(float)std::cos(ang), (float)std::sin(ang)});
      }
    for (int a4 = 0; a4 < 4; ++a4)
      for (int cc = 0; cc < 16; ++cc) {
        const double ang = -2.0 * M_PI * (double)(a4 * cc) / 64.0;
        tw.push_back(cf{(float)std::cos(ang), (float)std::sin(ang)});
      }
    HIPCHK(hipMemcpy(eng->dTw, tw.data(), tw.size() * sizeof(cf), hipMemcpyHostToDevice));
  }
  for (auto& cl : eng->classes) {
    HIPCHK(dalloc(&cl.dev, cl.host.size()));
    HIPCHK(dalloc(&cl.devIds, cl.ids.size()));
    HIPCHK(hipMemcpy(cl.dev, cl.host.data(), cl.host.size() * sizeof(FamNode), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(cl.devIds, cl.ids.data(), cl.ids.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  {
    // split solves for the GEVD of the lane classes D 9..12 and the lane-grid
    // classes (DANSE_LANE_SPLIT=1 turns them on)
    const char* sp = std::getenv("DANSE_LANE_SPLIT");
    const bool on = c->gevd && (sp && std::atoi(sp) != 0);
    for (auto& cl : eng->classes) cl.split = on && class_split(cl.DMAX) && (cl.G == 1 || cl.DMAX > kLaneMaxD);
    // the lean solves of the 8 x 8 grid classes with the C cache (not with
    // split solves, whose solving items run on the SM = 2 variant)
    for (auto& cl : eng->classes) {
      cl.lean = !cl.split && eng->cStride > 0 && eng->liStride > 0 && class_grid(cl.DMAX) == 8 && !std::getenv("DANSE_NO_LEAN");
      if (cl.lean) {
        bool any = false;
        for (const auto& fn : cl.host) any = any || fn.cOff >= 0;
        cl.lean = any;
      }
      if (cl.lean) {
        // (the noise-frame variant moves the float64 factor by rank one,
        // li_rank1_2d, which needs beta > 0 -- as update_kernel_2d's choice)
        cl.leanNoise = !std::getenv("DANSE_NO_LEAN_NOISE");
        for (int i = 0; i < S * K; ++i) cl.leanNoise = cl.leanNoise && c->beta[i] > 0.0;
        HIPCHK(dalloc(&cl.dFbList, (size_t)S * cl.host.size() * F));
        HIPCHK(dalloc(&cl.dFbCount, (size_t)R + 1));   // (+1: fallback_kernel_2d's done counter)
        HIPCHK(hipMemset(cl.dFbCount, 0, ((size_t)R + 1) * sizeof(int)));
      }
    }
    if (int rc = build_split_lists(eng, c->flags)) return rc;
  }
  if (!eng->wideIds.empty()) {
    int dw = 0;
    for (int id : eng->wideIds) dw = std::max(dw, eng->fns[id].D);
    eng->wideChunk = wide::chunk_for(dw, (long long)S * F);
    HIPCHK(dalloc(&eng->wideWork, (size_t)eng->wideChunk * wide::work_elems(dw)));
    HIPCHK(dalloc(&eng->dWideIds, eng->wideIds.size()));
    HIPCHK(hipMemcpy(eng->dWideIds, eng->wideIds.data(), eng->wideIds.size() * sizeof(int), hipMemcpyHostToDevice));
    build_wide_lists(eng, c->flags);
  }
  {
    // the gate's [D][D + 1] complex-double matrix in dynamic LDS above 64 KiB;
    // above kGateMaxD the packed lower triangle in a global workspace
    // (gate_wide_kernel: 512 (candidate, bin) workgroups per chunk)
    int dmax = 0;
    for (const auto& x : eng->fns) dmax = std::max(dmax, x.D);
    if (dmax > kGateMaxD) {
      eng->gateWorkItems = 512;
      HIPCHK(dalloc(&eng->gateWork, (size_t)eng->gateWorkItems * dmax * (dmax + 1) / 2));
    } else {
      const size_t lds = (size_t)dmax * (dmax + 1) * sizeof(cd);
      if (lds > 65536)
        HIPCHK(hipFuncSetAttribute((const void*)gate_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    }
  }
  const size_t MT = (size_t)eng->MT;
  HIPCHK(dalloc(&eng->Yspec, 2 * S * MT * F));
  HIPCHK(dalloc(&eng->Zspec, (size_t)2 * K * S * F));
  if (c->cEnd) {
    for (int i = 0; i < R * K; ++i)
      if (c->cEnd[i] < 0 || c->cEnd[i] > c->T + c->N) return fail(eng, "cEnd outside the signal");
    std::vector<int> chanNode;
    for (int q = 0; q < K; ++q)
      for (int m = 0; m < eng->M[q]; ++m) chanNode.push_back(q);
    HIPCHK(dalloc(&eng->dCEnd, (size_t)R * K));
    HIPCHK(hipMemcpy(eng->dCEnd, c->cEnd, (size_t)R * K * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(dalloc(&eng->dChanNode, MT));
    HIPCHK(hipMemcpy(eng->dChanNode, chanNode.data(), MT * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(dalloc(&eng->Cspec, (size_t)2 * S * MT * F));
  }
  if (c->cPhase) {
    HIPCHK(dalloc(&eng->dCPhase, (size_t)R * K * MT));
    HIPCHK(hipMemcpy(eng->dCPhase, c->cPhase, (size_t)R * K * MT * sizeof(double), hipMemcpyHostToDevice));
  }
  HIPCHK(dalloc(&eng->zPrev, (size_t)S * K * c->N));
  HIPCHK(dalloc(&eng->zStream, (size_t)S * K * eng->zLen));
  if (c->fsTab) {
    HIPCHK(dalloc(&eng->dFsTab, eng->fsTab.size()));
    HIPCHK(hipMemcpy(eng->dFsTab, eng->fsTab.data(), eng->fsTab.size() * sizeof(int), hipMemcpyHostToDevice));
    if (c->rawStreams) {
      if (!c->cEnd) return fail(eng, "rawStreams needs cEnd (the consumed raw stream ends)");
      HIPCHK(dalloc(&eng->rawStream, (size_t)S * eng->MT * eng->zLen));
    }
    HIPCHK(dalloc(&eng->dFsEv, std::max<size_t>(eng->fsEv.size(), 1)));
    if (!eng->fsEv.empty())
      HIPCHK(hipMemcpy(eng->dFsEv, eng->fsEv.data(), eng->fsEv.size() * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(dalloc(&eng->wIR, (size_t)S * K * eng->Mmax * tzc::kA));
    // sn[i] = sum_n f[n] h[n + i - N + 1] / (N Ns)  (dist_fct_approx with R = Ns)
    std::vector<float> sn(tzc::kA);
    for (int i = 0; i < tzc::kA; ++i) {
      const int tau = i - (c->N - 1);
      double acc = 0.0;
      for (int n = std::max(0, -tau); n < std::min(c->N, c->N - tau); ++n)
        acc += (double)c->winSynthesis[n] * (double)c->winAnalysis[n + tau];
      sn[i] = (float)(acc / ((double)c->N * (double)c->Ns));
    }
    HIPCHK(dalloc(&eng->dSn, (size_t)tzc::kA));
    HIPCHK(hipMemcpy(eng->dSn, sn.data(), sn.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  HIPCHK(dalloc(&eng->Ryy, (size_t)S * eng->scmStride));
  HIPCHK(dalloc(&eng->Rnn, (size_t)S * eng->scmStride));
  HIPCHK(dalloc(&eng->wHist, (size_t)S * eng->wStride));
  HIPCHK(dalloc(&eng->wExtHist, (size_t)S * eng->wExtStride));
  HIPCHK(dalloc(&eng->wExtTarget, (size_t)S * eng->tgtStride));
  HIPCHK(dalloc(&eng->dhat, (size_t)kMaxFam * S * K * R * F));
  HIPCHK(dalloc(&eng->d, (size_t)kMaxFam * S * K * c->T));
  HIPCHK(dalloc(&eng->diag, (size_t)S * K * kMaxFam));
  if (eng->liStride > 0) HIPCHK(dalloc(&eng->liCache, (size_t)S * eng->liStride));
  if (c->gevd && eng->liStride > 0) {
    for (auto& cl : eng->classes) {
      if (cl.G != 1) continue;
      const long long blocks = ((long long)S * (long long)cl.host.size() * F + 63) / 64;
      // (whole 1 KiB DMA pieces per block: kernels_lane.hpp lr_rows)
      HIPCHK(dalloc(&cl.liLane, (size_t)blocks * 64 * ((cl.DMAX * (cl.DMAX + 1) / 2 + cl.DMAX + 1) & ~1)));
    }
  }
  if (eng->vStride > 0) HIPCHK(dalloc(&eng->vCache, (size_t)S * eng->vStride));
  if (eng->vStride > 0) HIPCHK(dalloc(&eng->lzStats, (size_t)2 * R * kLzSlots));
  if (c->desSigConv) {
    // (the centralised / SSBC vectors' first M_k channels under SRO clocks
    // come from the receivers' raw buffers: not on this path)
    if (c->cEnd) return fail(eng, "desSigProcessingType conv with centralised / SSBC estimates under SRO clocks");
    eng->desConv = 1;
    HIPCHK(dalloc(&eng->convIR, (size_t)S * eng->fns.size() * eng->Mmax * tzc::kA));
    std::vector<float> sn(tzc::kA);
    for (int i = 0; i < tzc::kA; ++i) {
      const int tau = i - (c->N - 1);
      double acc = 0.0;
      for (int n = std::max(0, -tau); n < std::min(c->N, c->N - tau); ++n)
        acc += (double)c->winSynthesis[n] * (double)c->winSynthesis[n + tau];
      sn[i] = (float)(acc / ((double)c->N * (double)c->Ns));
    }
    HIPCHK(dalloc(&eng->dSnConv, (size_t)tzc::kA));
    HIPCHK(hipMemcpy(eng->dSnConv, sn.data(), sn.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  if (const char* tr = std::getenv("DANSE_UPDATE_TRACE")) {
    // (upper bound: one wave per (scene, family-node, bin))
    eng->updTraceRound = std::atoi(tr);
    eng->resTraceBytes = (size_t)S * eng->fns.size() * F * (kStampN + 1) * sizeof(unsigned long long);
    HIPCHK(hipMalloc((void**)&eng->resTrace, eng->resTraceBytes));
    HIPCHK(hipMemset(eng->resTrace, 0, eng->resTraceBytes));
  }
  if (eng->l64Stride > 0) HIPCHK(dalloc(&eng->l64Cache, (size_t)S * eng->l64Stride));
  if (eng->cStride > 0) HIPCHK(dalloc(&eng->cCache, (size_t)S * eng->cStride));
  if (c->dxcp) {
    if (c->cohDrift) return fail(eng, "DXCP-PhaT and CohDrift estimation are exclusive");
    if (c->fsTab) return fail(eng, "DXCP-PhaT estimation runs on wholeChunk broadcasts");
    if (kDxFrame % c->Ns) return fail(eng, "DXCP-PhaT frames need Ns dividing 2048");
    eng->dxcpOn = 1;
    eng->cdComp = c->cdCompensate;
    const size_t P = (size_t)S * (c->k1 - c->k0) * (K - 1);
    const size_t nq = (size_t)S * K * (K - 1);
    HIPCHK(dalloc(&eng->dxFrames, P * 2 * kDxFrame));
    HIPCHK(dalloc(&eng->dxOut, P * 2));
    HIPCHK(dalloc(&eng->dxEst, (size_t)S * K * K));
    HIPCHK(dalloc(&eng->cdPhase, (size_t)S * K * K));
    HIPCHK(dalloc(&eng->cdEst, nq * R));
    HIPCHK(dalloc(&eng->cdRes, nq * R));
    HIPCHK(hipMemset(eng->cdEst, 0, nq * R * sizeof(double)));
    HIPCHK(hipMemset(eng->cdRes, 0, nq * R * sizeof(double)));
    if (danse_dxcp_create((int)P, device, &eng->dx) != 0)
      return fail(eng, std::string("DXCP estimator: ") + danse_dxcp_last_error(nullptr));
  }
  if (c->cohDrift) {
    if (c->cdSegLength < 1 || c->cdEvery < 1 || c->cdStart < c->cdSegLength) return fail(eng, "bad CohDrift parameters");
    eng->cohDrift = 1;
    eng->cdLd = c->cdSegLength; eng->cdStart = c->cdStart; eng->cdEvery = c->cdEvery; eng->cdComp = c->cdCompensate;
    eng->cdNIter = c->cdNIter; eng->cdAlpha = c->cdAlpha; eng->cdAlphaEps = c->cdAlphaEps;
    if (c->cohDrift == 2) {
      if (!c->cdFlagWin) return fail(eng, "CohDrift open loop needs cdFlagWin");
      eng->cdOpen = 1;
      HIPCHK(dalloc(&eng->cdFlagWin, (size_t)R * K * K));
      HIPCHK(hipMemcpy(eng->cdFlagWin, c->cdFlagWin, (size_t)R * K * K * sizeof(double), hipMemcpyHostToDevice));
    } else if (c->cohDrift != 1) {
      return fail(eng, "cohDrift: 1 closed loop, 2 open loop");
    }
    const size_t nq = (size_t)S * K * (K - 1);
    HIPCHK(dalloc(&eng->cdRing, (size_t)(c->cdSegLength + 1) * nq * F));
    HIPCHK(dalloc(&eng->cdAvg, nq * F));
    HIPCHK(dalloc(&eng->cdPhase, (size_t)S * K * K));
    HIPCHK(dalloc(&eng->cdEst, nq * R));
    HIPCHK(dalloc(&eng->cdRes, nq * R));
  }
  HIPCHK(hipMemset(eng->Yspec, 0, 2 * S * MT * F * sizeof(cf)));
  HIPCHK(hipMemset(eng->Zspec, 0, (size_t)2 * K * S * F * sizeof(cf)));
  HIPCHK(hipMemset(eng->zPrev, 0, (size_t)S * K * c->N * sizeof(float)));
  HIPCHK(hipMemset(eng->zStream, 0, (size_t)S * K * eng->zLen * sizeof(float)));
  HIPCHK(hipMemset(eng->dhat, 0, (size_t)kMaxFam * S * K * R * F * sizeof(cf)));
  HIPCHK(hipMemset(eng->d, 0, (size_t)kMaxFam * S * K * c->T * sizeof(float)));
  HIPCHK(hipMemset(eng->diag, 0, (size_t)S * K * kMaxFam * sizeof(int)));
  HIPCHK(hipMemset(eng->Ryy, 0, (size_t)S * eng->scmStride * sizeof(cf)));
  HIPCHK(hipMemset(eng->Rnn, 0, (size_t)S * eng->scmStride * sizeof(cd)));
  HIPCHK(hipMemset(eng->wHist, 0, (size_t)S * eng->wStride * sizeof(cf)));
  HIPCHK(hipMemset(eng->wExtHist, 0, (size_t)S * eng->wExtStride * sizeof(cf)));

  // ---- initial state: host arrays are per family-node over ALL K nodes
  // (family-major); keep device copies so that danse_engine_reset() can
  // re-initialise the state on a stream.
  {
    std::vector<cf> w0h;
    std::vector<cd> scmh;
    long long w0Off = 0, scmInOff = 0;
    eng->scmPerBin = c->scmInitPerBin ? 1 : 0;
    const long long nSlice = eng->scmPerBin ? F : 1;
    for (int fam = 0; fam < kMaxFam; ++fam) {
      if (!((eng->families >> fam) & 1)) continue;
      for (int k = 0; k < K; ++k) {
        int D = (fam == DANSE_FAM_LOCAL) ? eng->M[k] : (fam == DANSE_FAM_CENTR ? (int)MT : eng->M[k] + K - 1);
        for (auto& x : eng->fns) {
          if (x.fam == fam && x.k == k) {
            eng->initW0Off.push_back((long long)w0h.size());
            eng->initScmOff.push_back((long long)scmh.size());
            for (long long e = 0; e < (long long)F * D; ++e)
              w0h.push_back(c->w0 ? cf{c->w0[2 * (w0Off + e)], c->w0[2 * (w0Off + e) + 1]} : cf{0.0f, 0.0f});
            for (long long e = 0; e < nSlice * D * D; ++e)
              scmh.push_back(c->scmInit ? cd{c->scmInit[2 * (scmInOff + e)], c->scmInit[2 * (scmInOff + e) + 1]}
                                        : cd{0.0, 0.0});
          }
        }
        w0Off += (long long)F * D;
        scmInOff += nSlice * D * D;
      }
    }
    std::vector<cf> exth, tgth;
    long long eOff = 0;
    for (int k = 0; k < K; ++k) {
      for (long long e = 0; e < (long long)F * eng->M[k]; ++e) {
        exth.push_back(c->wExt0 ? cf{c->wExt0[2 * (eOff + e)], c->wExt0[2 * (eOff + e) + 1]} : cf{0.0f, 0.0f});
        tgth.push_back(c->wExtTarget0 ? cf{c->wExtTarget0[2 * (eOff + e)], c->wExtTarget0[2 * (eOff + e) + 1]}
                                      : cf{0.0f, 0.0f});
      }
      eOff += (long long)F * eng->M[k];
    }
    eng->tgtOff = tgtOff;
    HIPCHK(dalloc(&eng->dW0, w0h.size()));
    HIPCHK(dalloc(&eng->dScm0, scmh.size()));
    HIPCHK(dalloc(&eng->dExt0, exth.size()));
    HIPCHK(dalloc(&eng->dTgt0, tgth.size()));
    HIPCHK(hipMemcpy(eng->dW0, w0h.data(), w0h.size() * sizeof(cf), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(eng->dScm0, scmh.data(), scmh.size() * sizeof(cd), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(eng->dExt0, exth.data(), exth.size() * sizeof(cf), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(eng->dTgt0, tgth.data(), tgth.size() * sizeof(cf), hipMemcpyHostToDevice));
    eng->extSrcOff.assign(K, 0);
    long long acc = 0;
    for (int k = 0; k < K; ++k) { eng->extSrcOff[k] = acc; acc += (long long)F * eng->M[k]; }
    HIPCHK(dalloc(&eng->dFnAll, eng->fns.size()));
    HIPCHK(hipMemcpy(eng->dFnAll, eng->fns.data(), eng->fns.size() * sizeof(FamNode), hipMemcpyHostToDevice));
    HIPCHK(dalloc(&eng->dInitW0Off, eng->fns.size()));
    HIPCHK(dalloc(&eng->dInitScmOff, eng->fns.size()));
    HIPCHK(hipMemcpy(eng->dInitW0Off, eng->initW0Off.data(), eng->fns.size() * sizeof(long long), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(eng->dInitScmOff, eng->initScmOff.data(), eng->fns.size() * sizeof(long long),
                     hipMemcpyHostToDevice));
    HIPCHK(dalloc(&eng->dExtSrcOff, K));
    HIPCHK(dalloc(&eng->dTgtOff, K));
    HIPCHK(hipMemcpy(eng->dExtSrcOff, eng->extSrcOff.data(), K * sizeof(long long), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(eng->dTgtOff, tgtOff.data(), K * sizeof(long long), hipMemcpyHostToDevice));
  }
  {
    // the prefix fast-forward: synchronous wholeChunk runs whose spectra the
    // recursion reads straight (no lags, phases, raw frames), no per-round
    // state beside the SCMs (CohDrift, DXCP, T(z) conv), the size classes'
    // packed SCMs (no wide class, no split solves, the recursion-only
    // variants on) -- DANSE_NO_FF=1: off
    bool ok = !std::getenv("DANSE_NO_FF") && !eng->noRO && !eng->dZLag && !eng->dZPhase && !eng->dCEnd &&
              !eng->dCPhase && !eng->cohDrift && !eng->dxcpOn && !eng->dFsTab && !eng->desConv &&
              eng->wideIds.empty() && eng->ffPraw > 0;
    for (const auto& cl : eng->classes) ok = ok && !cl.split;
    for (const auto& fn : eng->fns) ok = ok && (fn.packed == 1 || fn.packed == 2) && fn.D <= 64;
    // the histories' byte budget (DANSE_FF_MB, default 4096 MB): a longer
    // prefix is cut to the rounds that fit, the rest run per round
    const size_t perRound = ((size_t)S * eng->MT * F + (size_t)K * S * F) * sizeof(cf);
    const char* fb = std::getenv("DANSE_FF_MB");
    const size_t budget = (size_t)(fb ? std::max(0, std::atoi(fb)) : 4096) << 20;
    const int fit = (int)std::min<size_t>((size_t)eng->ffPraw, budget / perRound);
    if (ok && fit > 0) {
      eng->ffAlloc = fit;
      HIPCHK(dalloc(&eng->yHist, (size_t)eng->ffAlloc * S * eng->MT * F));
      HIPCHK(dalloc(&eng->zHist, (size_t)eng->ffAlloc * K * S * F));
      eng->ffOk = true;
      eng->ffP = std::min(eng->ffPraw, eng->ffAlloc);
    }
  }
  {
    int rc = danse_engine_reset(eng, nullptr);
    if (rc) return rc;
  }
  HIPCHK(hipDeviceSynchronize());
  *out = eng;
  return 0;
}

void danse_engine_destroy(danse_engine* eng) {
  if (!eng) return;
  (void)hipSetDevice(eng->dev);
  if (eng->graphExec) (void)hipGraphExecDestroy(eng->graphExec);
  void* ptrs[] = {eng->dM, eng->dBase, eng->dBcEnd, eng->dUpEnd, eng->dChan, eng->dFlags, eng->dZLag, eng->dZPhase,
                  eng->dBeta, eng->dBetaExt,
                  eng->dhA, eng->dhS, eng->dNorm, eng->dTw, eng->dWExtNodeOff, eng->Yspec,
                  eng->ownZspec ? eng->Zspec : nullptr, eng->Ryy,
                  eng->Rnn, eng->wHist, eng->wExtHist, eng->wExtTarget, eng->dhat, eng->zPrev, eng->zStream, eng->d,
                  eng->diag, eng->dW0, eng->dScm0, eng->dExt0, eng->dTgt0, eng->dFnAll, eng->dInitW0Off,
                  eng->dInitScmOff, eng->dExtSrcOff, eng->dTgtOff, eng->dFsTab, eng->wIR, eng->dSn, eng->liCache,
                  eng->dGateCand, eng->dGateVerdict, eng->cdRing, eng->cdAvg, eng->cdPhase, eng->cdEst,
                  eng->cdRes, eng->dCEnd, eng->Cspec, eng->dChanNode, eng->dCPhase, eng->dxFrames, eng->dxOut,
                  eng->dxEst, eng->resYB, eng->resYU, eng->resZall, eng->resZhat, eng->resRyyG, eng->resRnnG,
                  eng->resUFlag, eng->resZFlag, eng->resGateRound, eng->resDanseFni, eng->resErr, eng->resFams,
                  eng->resFrames, eng->resChanNode, eng->resTrace, eng->condHist, eng->dxRecFrames,
                  eng->dxRecOut, eng->dFsEv, eng->rawStream, eng->vCache, eng->l64Cache, eng->lzStats,
                  eng->dWideIds, eng->wideWork, eng->convIR, eng->dSnConv, eng->cCache, eng->yHist, eng->zHist,
                  eng->cdFlagWin, eng->gateWork};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (eng->dx) danse_dxcp_destroy(eng->dx);
  for (auto& cl : eng->classes) {
    if (cl.dev) (void)hipFree(cl.dev);
    if (cl.devIds) (void)hipFree(cl.devIds);
    if (cl.dSolveItems) (void)hipFree(cl.dSolveItems);
    if (cl.liLane) (void)hipFree(cl.liLane);
    if (cl.dCreItems) (void)hipFree(cl.dCreItems);
    if (cl.dCnItems) (void)hipFree(cl.dCnItems);
    if (cl.dFbList) (void)hipFree(cl.dFbList);
    if (cl.dFbCount) (void)hipFree(cl.dFbCount);
  }
  delete eng;
}

int danse_engine_set_inputs(danse_engine* eng, const float* yDev) {
  if (!eng || !yDev) return fail(eng, "null argument");
  eng->y = yDev;
  return 0;
}

static BcastArgs make_bcast(danse_engine* e, int r, int synth, int bc) {
  BcastArgs a{};
  a.S = e->S; a.K = e->K; a.MT = e->MT; a.T = e->T; a.N = e->N; a.Ns = e->Ns; a.F = e->F; a.R = e->R;
  a.r = r; a.k0 = e->k0; a.k1 = e->k1; a.families = e->families; a.doSynth = synth; a.doBcast = bc;
  a.M = e->dM; a.base = e->dBase; a.bcEnd = e->dBcEnd; a.upEnd = e->dUpEnd; a.y = e->y;
  a.Yspec = e->Yspec; a.Zspec = e->Zspec; a.zPrev = e->zPrev; a.zStream = e->zStream;
  a.wExtHist = e->wExtHist; a.wExtNodeOff = e->dWExtNodeOff; a.wExtStride = e->wExtStride;
  a.wExtHistory = e->keepHistory; a.dhat = e->dhat; a.d = e->d; a.hA = e->dhA; a.hS = e->dhS; a.normVal = e->dNorm;
  a.tw = e->dTw + e->N;
  a.dbg = e->bcastAblate;
  a.zLen = e->zLen;
  a.fsTab = e->dFsTab;
  a.cEnd = e->dCEnd; a.Cspec = e->Cspec; a.rawStream = e->rawStream; a.zChunk = e->zChunk;
  a.zMask = ~0u;
  a.zOnly = 0;
  a.foreign = e->foreign;
  return a;
}

static UpdateArgs make_update(danse_engine* e, int r) {
  UpdateArgs a{};
  a.S = e->S; a.K = e->K; a.MT = e->MT; a.F = e->F; a.R = e->R; a.r = r;
  a.chanList = e->dChan; a.flags = e->dFlags; a.Yspec = e->Yspec; a.Zspec = e->Zspec;
  a.zLag = e->dZLag; a.zPhase = e->dZPhase;
  a.Ryy = e->Ryy; a.Rnn = e->Rnn; a.scmStride = e->scmStride;
  a.wHist = e->wHist; a.wStride = e->wStride;
  a.wHistory = e->keepHistory; a.wExtHist = e->wExtHist; a.wExtStride = e->wExtStride; a.wExtHistory = e->keepHistory;
  a.wExtTarget = e->wExtTarget; a.tgtStride = e->tgtStride; a.dhat = e->dhat; a.beta = e->dBeta;
  a.betaExt = e->dBetaExt; a.alphaExt = e->alphaExt; a.gevd = e->gevd; a.rank = e->rank; a.diag = e->diag;
  a.liCache = e->liCache; a.liStride = e->liStride;
  a.vCache = e->vCache; a.vStride = e->vStride;
  a.l64Cache = e->l64Cache; a.l64Stride = e->l64Stride;
  a.cCache = e->cCache; a.cStride = e->cStride;
  a.lzStats = e->lzStats;
  a.cdPhase = e->cdPhase;
  a.Cspec = e->Cspec; a.chanNode = e->dChanNode; a.cPhase = e->dCPhase;
  a.nodeMask = ~0u;
  return a;
}

// mask: the nodes updated by this launch; full: the round's last update
// launch (its per-round extras run)
// ---- desSigProcessingType 'conv' (get_desired_sig_chunk, d_base.py:
// 2085-2100; get_desired_signal, d_classes.py:2623-2709): for every
// family-node, the IRs dist_fct_approx(w[r + 1][:, m], win_s, win_s, Ns) of
// the first M_k filter columns (one wave each, tzconv.hpp ir_wave), then the
// last Ns samples of their convolutions with the first M_k channels of the
// family's update frame (yTD = yTilde[k][:, i, :nLocalMic[k]]), idDesired =
// 2N - 1 - Ns .. 2N - 2 (one below the broadcast chunks' indices), summed
// over m into d[end - Ns, end); dhat is NaN (dhatCurr = None).
__global__ void __launch_bounds__(256) conv_ir_kernel(const UpdateArgs a, const FamNode* fns, int nFN, int Mmax,
                                                      const cf* tw, const float* snc, float* irOut) {
  __shared__ cf lds[4][wfft::kLdsElems];
  const int wv = threadIdx.x >> 6;
  const int item = blockIdx.x * 4 + wv;
  if (item >= a.S * nFN * Mmax) return;
  const int m = item % Mmax;
  const int fni = (item / Mmax) % nFN;
  const int s = item / (nFN * Mmax);
  const FamNode d = fns[fni];
  if (m >= d.M || !node_in(a.nodeMask, d.k)) return;
  const int slotNext = a.wHistory ? a.r + 1 : ((a.r + 1) & 1);
  const cf* w = a.wHist + (long long)s * a.wStride + d.wOff + (long long)slotNext * a.F * d.D + m;
  float* o = irOut + (((long long)s * nFN + fni) * Mmax + m) * tzc::kA;
  tzc::ir_wave(lds[wv], tw, snc, [&](int f) { return w[(long long)f * d.D]; }, [&](int t, float v) { o[t] = v; });
}

__global__ void __launch_bounds__(tzc::kThr) conv_d_kernel(const UpdateArgs a, const FamNode* fns, int nFN, int Mmax,
                                                           const int* upEnd, const float* y, int T, int N, int Ns,
                                                           const float* ir, float* d) {
  __shared__ tzc::ConvLds sm;
  const int fni = blockIdx.x % nFN;
  const int s = blockIdx.x / nFN;
  const FamNode fn = fns[fni];
  if (!node_in(a.nodeMask, fn.k)) return;
  const int r = a.r, K = a.K, F = a.F;
  const int end = upEnd[r * K + fn.k];
  const float* irb = ir + ((long long)s * nFN + fni) * Mmax * tzc::kA;
  float* dd = d + (((long long)fn.fam * a.S + s) * K + fn.k) * T;
  const int* ch = a.chanList + fn.chanOff;   // the family vector's first M_k channels (all < MT here)
  tzc::conv_block(
      sm, fn.M, Ns,
      [&](int q, int m) { return y[((long long)s * a.MT + ch[m]) * T + min(max(end - N + q, 0), T - 1)]; },
      [&](int q, int) { return end - N + q >= 0 && end - N + q < T; },
      [&](int i, int m) { return irb[(long long)m * tzc::kA + i]; },
      [&](int e, float v) {
        const int idx = end - Ns + e;
        if (idx >= 0 && idx < T) dd[idx] = v;
      },
      -1);
  const float qn = __builtin_nanf("");
  for (int f = threadIdx.x; f < F; f += blockDim.x)
    a.dhat[((((long long)fn.fam * a.S + s) * K + fn.k) * a.R + r) * F + f] = cf{qn, qn};
}

static void launch_conv(danse_engine* e, int r, hipStream_t st, unsigned mask) {
  UpdateArgs a = make_update(e, r);
  a.nodeMask = mask;
  const int nFN = (int)e->fns.size();
  const int items = e->S * nFN * e->Mmax;
  hipLaunchKernelGGL(conv_ir_kernel, dim3((items + 3) / 4), dim3(256), 0, st, a, e->dFnAll, nFN, e->Mmax,
                     e->dTw + e->N, e->dSnConv, e->convIR);
  hipLaunchKernelGGL(conv_d_kernel, dim3(e->S * nFN), dim3(tzc::kThr), 0, st, a, e->dFnAll, nFN, e->Mmax, e->dUpEnd,
                     e->y, e->T, e->N, e->Ns, e->convIR, e->d);
}

static void launch_wide(danse_engine* e, int r, hipStream_t st, unsigned mask) {
  const int nW = (int)e->wideIds.size();
  UpdateArgs a = make_update(e, r);
  a.nodeMask = mask;
  const int S = e->S, F = e->F, K = e->K;
  hipLaunchKernelGGL(wide_rec_kernel, dim3(F, S * nW), dim3(kWideRecThr), 0, st, a, e->dFnAll, e->dWideIds, nW);
  for (int w = 0; w < nW; ++w) {
    const FamNode& fn = e->fns[e->wideIds[w]];
    if (!((mask >> fn.k) & 1u) || !e->wideSolve[(size_t)r * nW + w]) continue;
    const int D = fn.D;
    const int slotNext = e->keepHistory ? r + 1 : ((r + 1) & 1);
    wide::WideArgs wa{};
    wa.D = D; wa.rank = e->rank; wa.gevd = e->gevd; wa.F = F; wa.nItems = (long long)S * F; wa.layout = 2;
    wa.RyyD = e->Rnn + fn.scmOff + (long long)F * D * (D + 1) / 2; wa.Rnn = e->Rnn + fn.scmOff;
    wa.srcScene = e->scmStride; wa.srcBin = (long long)D * (D + 1) / 2;
    wa.nOut = 1; wa.refs[0] = fn.ref; wa.wOff[0] = fn.wOff + (long long)slotNext * F * D;
    wa.w = e->wHist; wa.wScene = e->wStride; wa.wBin = D;
    wa.work = e->wideWork;
    wa.flags = e->dFlags + ((size_t)r * S * kMaxFam + fn.fam) * K + fn.k;
    wa.flagStride = (long long)kMaxFam * K;
    const hipError_t le = wide::launch_wide_filters(wa, e->wideChunk, st);
    if (le != hipSuccess && e->launchErr == hipSuccess) e->launchErr = le;
  }
  hipLaunchKernelGGL(wide_tail_kernel, dim3(F, S * nW), dim3(64), 0, st, a, e->dFnAll, e->dWideIds, nW);
}

static int ff_prefix(const danse_engine* e) { return e->condEvery == 0 ? e->ffP : 0; }

// the prefix's recursion over every bin of every family-node (span.hpp)
static void launch_span(danse_engine* e, hipStream_t st) {
  for (auto& cl : e->classes) {
    SpanArgs a{};
    a.S = e->S; a.K = e->K; a.MT = e->MT; a.F = e->F; a.P = ff_prefix(e); a.nFN = (int)cl.host.size();
    a.flags = e->dFlags; a.fn = cl.dev; a.chanList = e->dChan; a.yHist = e->yHist; a.zHist = e->zHist;
    a.Ryy = e->Ryy; a.Rnn = e->Rnn; a.scmStride = e->scmStride; a.beta = e->dBeta;
    launch_span_class(cl.DMAX, a, (unsigned)(e->S * a.nFN * e->F), st);
  }
}

static void launch_update(danse_engine* e, int r, hipStream_t st, unsigned mask = ~0u, bool full = true) {
  if (!e->wideIds.empty()) launch_wide(e, r, st, mask);
  const bool ff = r < ff_prefix(e) && mask == ~0u && full;
  if (ff) {
    // this round's update-frame and fused spectra into the histories
    const size_t ny = (size_t)e->S * e->MT * e->F, nz = (size_t)e->K * e->S * e->F;
    const size_t n = ny + nz;
    const unsigned blocks = (unsigned)(n < (size_t)256 * 4096 ? (n + 255) / 256 : 4096);
    hipLaunchKernelGGL(ff_copy_kernel, dim3(blocks), dim3(256), 0, st, e->yHist + (size_t)r * ny,
                       e->Yspec + (size_t)((r + 1) & 1) * ny, ny, e->zHist + (size_t)r * nz,
                       e->Zspec + (size_t)(r & 1) * nz, nz);
  }
  for (auto& cl : e->classes) {
    UpdateArgs a = make_update(e, r);
    a.noRec = ff ? 1 : 0;
    a.nodeMask = mask;
    a.nFN = (int)cl.host.size();
    a.fn = cl.dev;
    a.famNodeId = cl.devIds;
    a.splitSolve = cl.split ? 1 : 0;
    a.liLane = cl.liLane;
    a.noSolve = (!e->noRO && (int)cl.anySolve.size() > r && !cl.anySolve[r]) ? 1 : 0;
    if (r == e->updTraceRound) a.stamps = e->resTrace;
    // the solves on the cached factor and C: update_kernel_2dc (whole-round
    // launches only; the fewSamples node-subset steps keep one kernel)
    const int nItems = e->S * (int)cl.host.size();
    const bool leanRound = cl.lean && mask == ~0u && (int)cl.creCount.size() > r;
    const int nCre = leanRound ? cl.creCount[r] : 0;
    const int nCn = leanRound ? cl.cnCount[r] : 0;
    a.leanOn = nCre > 0 ? 1 : 0;
    a.leanNoise = nCn > 0 ? 1 : 0;
    a.creItems = cl.dCreItems + (size_t)r * nItems;
    a.cnItems = cl.dCnItems + (size_t)r * nItems;
    a.fbList = cl.dFbList;
    a.fbCount = cl.dFbCount;
    if (nCre + nCn < nItems) launch_update_class(cl.DMAX, a, st);   // D > kMaxDMax rejected at create time
    if (nCre + nCn > 0) {
      // (one counter per round: each round's lean launch counts its own
      // failed warm solves, and its fallback launch zeroes the counter when
      // its last block is done)
      launch_lean_solve_class(cl.DMAX, a, nCre, nCn, std::min((nCre + nCn) * e->F, 256), st);
    }
    if (cl.split && cl.solveCount[r] > 0) {
      a.solveItems = cl.dSolveItems + (size_t)r * e->S * cl.host.size();
      launch_split_solve_class(cl.DMAX, a, cl.solveCount[r], st);
    }
  }
  if (e->desConv) launch_conv(e, r, st, mask);
  if (!full) return;
  if (e->condEvery > 0 && (r + 1) % e->condEvery == 0) {
    // (saved when i - last >= every, last starting at -1: d_classes.py:2128-2130)
    int dm = 1;
    for (const auto& fn : e->fns) dm = std::max(dm, fn.D);
    const size_t lds = (size_t)dm * (dm + 1) * sizeof(cd);
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)cond_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(cond_kernel, dim3(e->F, e->S * (int)e->fns.size()), dim3(64), lds, st, make_update(e, r),
                       e->dFnAll, (int)e->fns.size(), e->condHist);
  }
  if (e->cohDrift) {
    CohDriftArgs c{};
    c.S = e->S; c.K = e->K; c.MT = e->MT; c.F = e->F; c.r = r; c.ld = e->cdLd; c.start = e->cdStart;
    c.every = e->cdEvery; c.nIter = e->cdNIter; c.compensate = e->cdComp; c.alpha = e->cdAlpha;
    c.alphaEps = e->cdAlphaEps; c.Ns = (double)e->Ns; c.base = e->dBase; c.ring = e->cdRing; c.avgTail = e->cdAvg;
    c.phase = e->cdPhase; c.est = e->cdEst; c.res = e->cdRes; c.R = e->R;
    c.open = e->cdOpen; c.flagWin = e->cdFlagWin;
    c.k0 = e->k0; c.nOwn = e->k1 - e->k0;
    hipLaunchKernelGGL(cohdrift_kernel, dim3(e->S * c.nOwn * (e->K - 1)), dim3(kCdThreads), 0, st, make_update(e, r), c);
  }
  if (e->dxcpOn) {
    const int nOwn = e->k1 - e->k0;
    const int P = e->S * nOwn * (e->K - 1);
    const int every = kDxFrame / e->Ns;
    const int fed = ((r + 1) % every) == 0;
    if (fed) {
      hipLaunchKernelGGL(dxcp_gather_kernel, dim3(P), dim3(256), 0, st, make_update(e, r), e->dUpEnd, e->y, e->zStream,
                         e->zLen, e->T, e->Ns, e->dBase, e->ref, e->k0, nOwn, e->dxFrames);
      (void)danse_dxcp_process(e->dx, e->dxFrames, e->dxOut, st);
      const int feed = (r + 1) / every - 1;
      if (e->dxRecFrames && feed < e->dxRecFeeds) {
        // (kernel copies: this runs inside the engine's captured graph)
        (void)copy_async(e->dxRecFrames + (size_t)feed * P * 2 * kDxFrame, e->dxFrames,
                         (size_t)P * 2 * kDxFrame * sizeof(float), st);
        (void)copy_async(e->dxRecOut + (size_t)feed * P * 2, e->dxOut, (size_t)P * 2 * sizeof(double), st);
      }
    }
    hipLaunchKernelGGL(dxcp_round_kernel, dim3((P + 63) / 64), dim3(64), 0, st, e->S, e->K, e->k0, nOwn, r, e->R, fed,
                       e->cdComp, (double)e->Ns, e->dxOut, e->dxEst, e->cdPhase, e->cdEst, e->cdRes);
  }
}

// one CHUNK step: the T(z) IR refreshes and chunk appends of fsEv row `row`
static void launch_fs(danse_engine* e, int row, hipStream_t st) {
  FsArgs a{};
  a.S = e->S; a.K = e->K; a.MT = e->MT; a.T = e->T; a.N = e->N; a.F = e->F; a.r = row; a.k0 = e->k0; a.k1 = e->k1;
  a.Mmax = e->Mmax; a.ref = e->ref; a.keepHistory = e->keepHistory; a.zLen = e->zLen;
  a.M = e->dM; a.base = e->dBase; a.fsTab = e->dFsEv; a.y = e->y;
  a.wExtHist = e->wExtHist; a.wExtNodeOff = e->dWExtNodeOff; a.wExtStride = e->wExtStride;
  a.tw = e->dTw + e->N; a.sn = e->dSn; a.wIR = e->wIR; a.zStream = e->zStream; a.rawStream = e->rawStream;
  const int nOwn = e->k1 - e->k0;
  a.foreign = (e->foreign && e->rawStream) ? 1 : 0;
  bool refresh = false, chunk = false;
  for (int k = 0; k < e->K; ++k) {
    const int* t = &e->fsEv[((size_t)row * e->K + k) * DANSE_FS_FIELDS];
    const bool own = k >= e->k0 && k < e->k1;
    refresh = refresh || (own && t[DANSE_FS_IRSRC] >= 0);
    chunk = chunk || ((own || a.foreign) && t[DANSE_FS_LEN] > 0);
  }
  if (refresh) {
    const unsigned items = (unsigned)(e->S * nOwn * e->Mmax);
    hipLaunchKernelGGL(fs_ir_kernel, dim3((items + 3) / 4), dim3(256), 0, st, a);
  }
  if (chunk) hipLaunchKernelGGL(fs_chunk_kernel, dim3(e->S * (a.foreign ? e->K : nOwn)), dim3(tzc::kThr), 0, st, a);
}

// zMask: fewSamples senders whose z frame this launch analyses; zOnly: that
// analysis alone (no local-frame analyses, no estimate synthesis)
static void launch_bcast(danse_engine* e, int r, int synth, int bc, hipStream_t st, unsigned zMask = ~0u,
                         int zOnly = 0) {
  if (bc && r > 0 && r == ff_prefix(e)) launch_span(e, st);   // (before round r's gate and update)
  if (e->desConv) synth = 0;   // ('conv': conv_d_kernel writes the estimates after each update)
  if (!synth && !bc) return;
  BcastArgs a = make_bcast(e, r, synth, bc);
  a.zMask = zMask;
  a.zOnly = zOnly;
  const unsigned grid = (unsigned)(e->S * (e->foreign ? e->K : e->k1 - e->k0));
  if (bcast_waves(e->S, e->K) == 8) hipLaunchKernelGGL(bcast_kernel<8>, dim3(grid), dim3(512), 0, st, a);
  else hipLaunchKernelGGL(bcast_kernel<4>, dim3(grid), dim3(256), 0, st, a);
}

// the installed speculative gate candidates of round r (danse_engine_set_gate)
// whose node is in `mask`
// the gate checks of n candidates (GateCand) of filter dimensions up to dmax:
// gate_kernel_reg (one wave per (candidate, bin), the matrix in registers) up
// to kGateRegMaxD, gate_kernel (the matrix in LDS) up to kGateMaxD,
// gate_wide_kernel (one workgroup per (candidate, bin), the matrix in
// eng->gateWork, in chunks) above; DANSE_GATE_LDS=1: gate_kernel up to
// kGateMaxD (A/B)
// (DANSE_GATE_WAVE=1: the wave-per-bin kernels below also for D <= 12, A/B only)
static bool gate_wave() {
  static const bool v = std::getenv("DANSE_GATE_WAVE") != nullptr;
  return v;
}
static void launch_gate(danse_engine* eng, const UpdateArgs& a, const GateCand* cand, int n, int dmax, int* verdict,
                        hipStream_t s) {
  if (dmax <= kGateLaneMaxD - 1 && !gate_wave()) {
    const unsigned grid = (unsigned)(((long long)n * eng->F + 63) / 64);
#define DANSE_GATE_LANE(DM)                                                                                 \
  do {                                                                                                      \
    if (eng->scmPerBin)                                                                                     \
      hipLaunchKernelGGL((gate_kernel_lane<DM, true>), dim3(grid), dim3(64), 0, s, a, eng->dFnAll, cand, n,  \
                         eng->dInitScmOff, eng->dScm0, eng->scmPerBin, verdict);                            \
    else                                                                                                    \
      hipLaunchKernelGGL((gate_kernel_lane<DM, false>), dim3(grid), dim3(64), 0, s, a, eng->dFnAll, cand, n, \
                         eng->dInitScmOff, eng->dScm0, eng->scmPerBin, verdict);                            \
  } while (0)
    if (dmax <= 4) DANSE_GATE_LANE(4);
    else if (dmax <= 8) DANSE_GATE_LANE(8);
    else DANSE_GATE_LANE(11);
#undef DANSE_GATE_LANE
    return;
  }
  if (dmax <= kGateRegMaxD && !std::getenv("DANSE_GATE_LDS")) {
    const int ne = gate_reg_ne(dmax);
#define DANSE_GATE_REG(NE)                                                                                    \
  hipLaunchKernelGGL(gate_kernel_reg<NE>, dim3(eng->F, n), dim3(64), 0, s, a, eng->dFnAll, cand, eng->dInitScmOff, \
                     eng->dScm0, eng->scmPerBin, verdict)
    if (ne == 2) DANSE_GATE_REG(2);
    else if (ne == 4) DANSE_GATE_REG(4);
    else if (ne == 8) DANSE_GATE_REG(8);
    else DANSE_GATE_REG(13);
#undef DANSE_GATE_REG
    return;
  }
  if (dmax <= kGateMaxD || !eng->gateWork) {
    const size_t lds = (size_t)dmax * (dmax + 1) * sizeof(cd);
    hipLaunchKernelGGL(gate_kernel, dim3(eng->F, n), dim3(64), lds, s, a, eng->dFnAll, cand, eng->dInitScmOff,
                       eng->dScm0, eng->scmPerBin, verdict);
    return;
  }
  const long long items = (long long)n * eng->F;
  for (long long i0 = 0; i0 < items; i0 += eng->gateWorkItems) {
    const long long m = std::min(eng->gateWorkItems, items - i0);
    hipLaunchKernelGGL(gate_wide_kernel, dim3((unsigned)m), dim3(kGateWideThr), 0, s, a, eng->dFnAll, cand,
                       eng->dInitScmOff, eng->dScm0, eng->scmPerBin, verdict, i0, eng->gateWork);
  }
}

static void launch_gate_round(danse_engine* eng, int r, hipStream_t s, unsigned mask = ~0u) {
  if (eng->nGate > 0 && eng->gateOff[r + 1] > eng->gateOff[r]) {
    const int n = eng->gateOff[r + 1] - eng->gateOff[r];
    UpdateArgs a = make_update(eng, r);
    a.nodeMask = mask;
    launch_gate(eng, a, eng->dGateCand + eng->gateOff[r], n, eng->gateDmax[r], eng->dGateVerdict + eng->gateOff[r], s);
  }
}

// fewSamples: steps [i0, i1) of the step list (compile_rounds_fs)
static void run_fs_steps(danse_engine* e, int i0, int i1, hipStream_t st) {
  const unsigned all = (1u << e->K) - 1u;
  for (int i = i0; i < i1; ++i) {
    const int* x = &e->fsSteps[(size_t)i * DANSE_FS_STEP_FIELDS];
    const int ty = x[0], r = x[1];
    const unsigned mask = (unsigned)x[2];
    if (ty == DANSE_FS_STEP_CHUNK) {
      launch_fs(e, x[3], st);
    } else if (ty == DANSE_FS_STEP_BCAST) {
      launch_bcast(e, r, r > 0, 1, st, mask, 0);
    } else if (ty == DANSE_FS_STEP_ZAN) {
      launch_bcast(e, r, 0, 1, st, mask, 1);
    } else {
      // the round's per-round extras (condition numbers, SRO estimators) run
      // with its last update step
      unsigned upd = 0;
      for (int j = e->fsRoundStep[r]; j <= i; ++j) {
        const int* y = &e->fsSteps[(size_t)j * DANSE_FS_STEP_FIELDS];
        if (y[0] == DANSE_FS_STEP_UPDATE) upd |= (unsigned)y[2];
      }
      launch_gate_round(e, r, st, mask);
      launch_update(e, r, st, mask, upd == all);
    }
  }
}

// the first UPDATE step of round r (fewSamples)
static int fs_first_update(const danse_engine* e, int r) {
  for (int i = e->fsRoundStep[r]; i < e->fsRoundStep[r + 1]; ++i)
    if (e->fsSteps[(size_t)i * DANSE_FS_STEP_FIELDS] == DANSE_FS_STEP_UPDATE) return i;
  return e->fsRoundStep[r + 1];
}

int danse_engine_gate_launch(danse_engine* eng, int32_t r, void* stream) {
  if (!eng || !eng->y) return fail(eng, "inputs not set");
  if (r < 0 || r >= eng->R) return fail(eng, "round out of range");
  HIPCHK(hipSetDevice(eng->dev));
  hipStream_t st = (hipStream_t)stream;
  if (eng->nGate > 0 && r == 0) HIPCHK(fill_async(eng->dGateVerdict, 0xff, eng->nGate * sizeof(int), st));
  // (fewSamples: the checks run inside danse_engine_update, before each
  // update step of their node)
  if (!eng->dFsTab) launch_gate_round(eng, r, st);
  HIPCHK(hipGetLastError());
  return 0;
}

int danse_engine_bcast(danse_engine* eng, int32_t r, void* stream) {
  if (!eng || !eng->y) return fail(eng, "inputs not set");
  if (r < 0 || r >= eng->R) return fail(eng, "round out of range");
  HIPCHK(hipSetDevice(eng->dev));
  if (eng->dFsTab)
    run_fs_steps(eng, eng->fsRoundStep[r], fs_first_update(eng, r), (hipStream_t)stream);
  else
    launch_bcast(eng, r, r > 0, 1, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return 0;
}

int danse_engine_update(danse_engine* eng, int32_t r, void* stream) {
  if (!eng) return fail(eng, "null engine");
  if (r < 0 || r >= eng->R) return fail(eng, "round out of range");
  HIPCHK(hipSetDevice(eng->dev));
  if (eng->dFsTab)
    run_fs_steps(eng, fs_first_update(eng, r), eng->fsRoundStep[r + 1], (hipStream_t)stream);
  else
    launch_update(eng, r, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return take_launch_err(eng);
}

int danse_engine_run_steps(danse_engine* eng, int32_t s0, int32_t s1, void* stream) {
  if (!eng || !eng->y) return fail(eng, "inputs not set");
  if (!eng->dFsTab) return fail(eng, "step lists are for fewSamples engines");
  const int n = (int)(eng->fsSteps.size() / DANSE_FS_STEP_FIELDS);
  if (s0 < 0 || s1 > n || s0 > s1) return fail(eng, "bad step range");
  HIPCHK(hipSetDevice(eng->dev));
  run_fs_steps(eng, s0, s1, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return take_launch_err(eng);
}

int danse_engine_finish(danse_engine* eng, void* stream) {
  if (!eng) return fail(eng, "null engine");
  HIPCHK(hipSetDevice(eng->dev));
  launch_bcast(eng, eng->R, 1, 0, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return 0;
}

int danse_engine_run(danse_engine* eng, int32_t r0, int32_t r1, void* stream, int32_t graph) {
  if (!eng || !eng->y) return fail(eng, "inputs not set");
  if (r0 < 0 || r1 > eng->R || r0 >= r1) return fail(eng, "bad round range");
  HIPCHK(hipSetDevice(eng->dev));
  hipStream_t st = (hipStream_t)stream;
  auto seq = [&](hipStream_t s) {
    if (eng->nGate > 0 && r0 == 0) (void)fill_async(eng->dGateVerdict, 0xff, eng->nGate * sizeof(int), s);
    if (eng->dFsTab) {
      run_fs_steps(eng, eng->fsRoundStep[r0], eng->fsRoundStep[r1], s);
    } else {
      for (int r = r0; r < r1; ++r) {
        launch_bcast(eng, r, r > 0, 1, s);
        launch_gate_round(eng, r, s);
        launch_update(eng, r, s);
      }
    }
    if (r1 == eng->R) launch_bcast(eng, eng->R, 1, 0, s);
  };
  if (!graph) {
    seq(st);
    HIPCHK(hipGetLastError());
    return take_launch_err(eng);
  }
  if (!(eng->graphExec && eng->graphR0 == r0 && eng->graphR1 == r1)) {
    if (eng->graphExec) {
      (void)hipGraphExecDestroy(eng->graphExec);
      eng->graphExec = nullptr;
    }
    hipStream_t cap = st;
    bool own = false;
    if (cap == nullptr) {
      HIPCHK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
      own = true;
    }
    hipGraph_t g;
    HIPCHK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
    seq(cap);
    HIPCHK(hipStreamEndCapture(cap, &g));
    if (eng->launchErr != hipSuccess) {
      (void)hipGraphDestroy(g);
      if (own) (void)hipStreamDestroy(cap);
      return take_launch_err(eng);
    }
    HIPCHK(hipGraphInstantiate(&eng->graphExec, g, nullptr, nullptr, 0));
    HIPCHK(hipGraphDestroy(g));
    if (own) HIPCHK(hipStreamDestroy(cap));
    eng->graphR0 = r0;
    eng->graphR1 = r1;
  }
  HIPCHK(hipGraphLaunch(eng->graphExec, st));
  return 0;
}

// ---- the resident engine (resident.hpp) -----------------------------------
static int resident_prepare(danse_engine* eng, int& NB) {
  danse_engine* e = eng;
  if (e->k0 != 0 || e->k1 != e->K) return fail(e, "resident run: the engine must own every node");
  if (e->dFsTab) return fail(e, "resident run: wholeChunk broadcasts only");
  if (e->cohDrift || e->dxcpOn) return fail(e, "resident run: no CohDrift / DXCP estimation");
  if (e->dCEnd) return fail(e, "resident run: no centralised raw frames (cEnd)");
  if (!e->gevd) return fail(e, "resident run: GEVD filters only");
  if (2 * e->Ns != e->N || e->Ns > 512) return fail(e, "resident run: 50 % frame overlap (Ns = N / 2 = 512) only");
  int dmax = 1;
  for (const auto& fn : e->fns) {
    if (fn.packed == 1 || fn.D > 12) return fail(e, "resident run: filter dimensions <= 12 in grid storage (smallDGrid)");
    dmax = std::max(dmax, fn.D);
  }
  NB = 3;
  const int S = e->S, K = e->K, F = e->F, R = e->R, MT = e->MT;
  std::vector<int> up((size_t)R * K);
  HIPCHK(hipMemcpy(up.data(), e->dUpEnd, up.size() * sizeof(int), hipMemcpyDeviceToHost));
  for (int k = 0; k < K; ++k)
    for (int r = 1; r < R; ++r)
      if (up[(size_t)r * K + k] < up[(size_t)(r - 1) * K + k]) return fail(e, "resident run: update frames go backwards");
  if (!e->resYB) {
    const int nFN = (int)e->fns.size();
    std::vector<int> danseFni(K, -1), fams;
    for (int i = 0; i < nFN; ++i)
      if (e->fns[i].fam == DANSE_FAM_DANSE) danseFni[e->fns[i].k] = i;
    for (int f = 0; f < kMaxFam; ++f)
      if ((e->families >> f) & 1) fams.push_back(f);
    e->resNFam = (int)fams.size();
    HIPCHK(dalloc(&e->resYB, (size_t)R * S * MT * F));
    HIPCHK(dalloc(&e->resYU, (size_t)R * S * MT * F));
    HIPCHK(dalloc(&e->resZall, (size_t)(R + 1) * K * S * F));
    HIPCHK(dalloc(&e->resZhat, (size_t)S * K * F));
    HIPCHK(dalloc(&e->resRyyG, (size_t)S * e->scmStride));
    HIPCHK(dalloc(&e->resRnnG, (size_t)S * e->scmStride));
    HIPCHK(dalloc(&e->resUFlag, (size_t)S * nFN * ((F + res::kBins - 1) / res::kBins)));
    HIPCHK(dalloc(&e->resZFlag, (size_t)S * K));
    HIPCHK(dalloc(&e->resGateRound, (size_t)S * nFN));
    HIPCHK(dalloc(&e->resDanseFni, (size_t)K));
    HIPCHK(dalloc(&e->resErr, 1));
    HIPCHK(dalloc(&e->resFams, fams.size()));
    HIPCHK(dalloc(&e->resFrames, (size_t)e->resNFam * S * K * R * e->N));
    std::vector<int> chanNode;
    for (int q = 0; q < K; ++q)
      for (int m = 0; m < e->M[q]; ++m) chanNode.push_back(q);
    HIPCHK(dalloc(&e->resChanNode, (size_t)MT));
    HIPCHK(hipMemcpy(e->resChanNode, chanNode.data(), MT * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->resDanseFni, danseFni.data(), K * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->resFams, fams.data(), fams.size() * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(hipMemset(e->resErr, 0, sizeof(int)));
  }
  return 0;
}

static UpdateArgs make_update_resident(danse_engine* e, int r) {
  UpdateArgs a = make_update(e, r);
  a.Yall = e->resYU;
  a.zAll = 1;
  a.Zspec = e->resZall;
  return a;
}

int danse_engine_run_resident(danse_engine* eng, void* stream) {
  if (!eng || !eng->y) return fail(eng, "inputs not set");
  if (eng->desConv) return fail(eng, "resident run: WOLA estimates only (desSigProcessingType wola)");
  HIPCHK(hipSetDevice(eng->dev));
  int NB = 0;
  if (int rc = resident_prepare(eng, NB)) return rc;
  hipStream_t st = (hipStream_t)stream;
  const int S = eng->S, K = eng->K, F = eng->F, R = eng->R;
  const int nFN = (int)eng->fns.size();
  const int FG = (F + res::kBins - 1) / res::kBins;
  res::ResArgs ra{};
  ra.u = make_update_resident(eng, 0);
  ra.b = make_bcast(eng, 1, 0, 1);
  ra.fn = eng->dFnAll;
  ra.danseFni = eng->resDanseFni;
  ra.nFN = nFN; ra.FG = FG; ra.nZ = S * K; ra.R = R;
  ra.YB = eng->resYB;
  ra.zhat = eng->resZhat;
  ra.uFlag = eng->resUFlag;
  ra.zFlag = eng->resZFlag;
  ra.gateRound = eng->resGateRound;
  ra.RyyG = eng->resRyyG;
  ra.RnnG = eng->resRnnG;
  ra.err = eng->resErr;
  const int grid = ra.nZ + S * nFN * FG;
  if (std::getenv("DANSE_RESIDENT_TRACE")) {
    const size_t nb = (size_t)R * grid * 2 * sizeof(unsigned long long);
    if (eng->resTraceBytes != nb) {
      if (eng->resTrace) (void)hipFree(eng->resTrace);
      HIPCHK(hipMalloc((void**)&eng->resTrace, nb));
      eng->resTraceBytes = nb;
    }
    HIPCHK(fill_async(eng->resTrace, 0, nb, st));
    ra.trace = eng->resTrace;
  }
  int fits = 0;
  const int chk = resident_launch(NB, eng->rank == 1, ra, grid, st, true, &fits);
  if (chk < 0) return fail(eng, "resident run: occupancy query failed");
  if (chk > 0)
    return fail(eng, "resident run: " + std::to_string(grid) + " waves do not fit the device at once (" +
                         std::to_string(fits) + ")");
  // gate snapshot rounds per (scene, family-node)
  std::vector<int> gr((size_t)S * nFN, -1);
  for (auto& x : eng->gateHost) gr[(size_t)x.second.s * nFN + x.second.fni] = x.first;
  HIPCHK(hipMemcpyAsync(eng->resGateRound, gr.data(), gr.size() * sizeof(int), hipMemcpyHostToDevice, st));
  HIPCHK(fill_async(eng->resUFlag, 0, (size_t)S * nFN * FG * sizeof(unsigned), st));
  HIPCHK(fill_async(eng->resZFlag, 0, (size_t)S * K * sizeof(unsigned), st));
  HIPCHK(fill_async(eng->resErr, 0, sizeof(int), st));   // per run: a previous run's give-up does not stick
  HIPCHK(fill_async(eng->resZall, 0, (size_t)K * S * F * sizeof(cf), st));   // slot 0: before round 0
  if (eng->nGate > 0) HIPCHK(fill_async(eng->dGateVerdict, 0xff, eng->nGate * sizeof(int), st));
  // WOLA analyses of every round (inputs only)
  {
    BcastArgs b = make_bcast(eng, 0, 0, 1);
    resident_analysis(b, eng->resChanNode, eng->resYB, eng->resYU, st);
    HIPCHK(hipGetLastError());
  }
  // round 0's broadcast into slot 1
  {
    BcastArgs b = make_bcast(eng, 0, 0, 1);
    b.Zspec = eng->resZall + (size_t)K * S * F;
    // (four waves: the resident kernel's own broadcasts sum the fused spectra in that order)
    hipLaunchKernelGGL(bcast_kernel<4>, dim3((unsigned)(S * K)), dim3(256), 0, st, b);
    HIPCHK(hipGetLastError());
  }
  if (resident_launch(NB, eng->rank == 1, ra, grid, st, false, &fits) != 0) return fail(eng, "resident launch failed");
  // the speculative gate checks, on the snapshots of the candidates' rounds
  for (int r = 0; r < R && eng->nGate > 0; ++r) {
    if (eng->gateOff[r + 1] == eng->gateOff[r]) continue;
    const int n = eng->gateOff[r + 1] - eng->gateOff[r];
    const size_t lds = (size_t)eng->gateDmax[r] * (eng->gateDmax[r] + 1) * sizeof(cd);
    UpdateArgs a = make_update_resident(eng, r);
    a.Ryy = eng->resRyyG;
    a.Rnn = eng->resRnnG;
    hipLaunchKernelGGL(gate_kernel, dim3(F, n), dim3(64), lds, st, a, eng->dFnAll, eng->dGateCand + eng->gateOff[r],
                       eng->dInitScmOff, eng->dScm0, eng->scmPerBin, eng->dGateVerdict + eng->gateOff[r]);
  }
  // estimate synthesis of every round
  {
    BcastArgs b = make_bcast(eng, R, 1, 0);
    resident_synth(b, eng->resFams, eng->resNFam, eng->resFrames, st);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

int danse_engine_set_cond(danse_engine* eng, int32_t every) {
  if (!eng || every < 0) return fail(eng, "bad condition-number interval");
  if (every > 0 && !eng->wideIds.empty()) return fail(eng, "condition numbers above 64 channels are not supported");
  HIPCHK(hipSetDevice(eng->dev));
  if (eng->graphExec) {   // the captured run changes
    (void)hipGraphExecDestroy(eng->graphExec);
    eng->graphExec = nullptr;
  }
  eng->condEvery = every;
  if (every > 0 && !eng->condHist) {
    const size_t n = (size_t)eng->S * eng->fns.size() * eng->R * eng->F;
    HIPCHK(dalloc(&eng->condHist, n));
    std::vector<double> nan(n, std::nan(""));
    HIPCHK(hipMemcpy(eng->condHist, nan.data(), n * sizeof(double), hipMemcpyHostToDevice));
  }
  return 0;
}

int danse_engine_cond(danse_engine* eng, double* dst, size_t bytes) {
  if (!eng || !dst) return fail(eng, "null argument");
  if (!eng->condHist) return fail(eng, "condition numbers are not enabled (danse_engine_set_cond)");
  const size_t n = (size_t)eng->S * eng->fns.size() * eng->R * eng->F;
  if (bytes < n * sizeof(double)) return fail(eng, "destination too small");
  HIPCHK(hipSetDevice(eng->dev));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(dst, eng->condHist, n * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

// diagnostics: the DANSE_RESIDENT_TRACE wall-clock marks of the last
// resident run ([R][grid][2] uint64, 100 MHz), bytes = 0 if none
int danse_engine_resident_trace(danse_engine* eng, void* dst, size_t* bytes) {
  if (!eng || !bytes) return fail(eng, "null argument");
  if (dst && eng->resTrace) HIPCHK(hipMemcpy(dst, eng->resTrace, std::min(*bytes, eng->resTraceBytes), hipMemcpyDeviceToHost));
  *bytes = eng->resTraceBytes;
  return 0;
}

int danse_engine_resident_error(danse_engine* eng, int32_t* err, void* stream) {
  if (!eng || !err) return fail(eng, "null argument");
  *err = 0;
  if (!eng->resErr) return 0;
  HIPCHK(hipSetDevice(eng->dev));
  HIPCHK(hipMemcpyAsync(err, eng->resErr, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

int danse_engine_resident_set_error(danse_engine* eng, int32_t value) {
  if (!eng) return fail(eng, "null engine");
  if (!eng->resErr) return fail(eng, "no resident run prepared");
  HIPCHK(hipSetDevice(eng->dev));
  HIPCHK(hipMemcpy(eng->resErr, &value, sizeof(int), hipMemcpyHostToDevice));
  return 0;
}

int danse_engine_dxcp_record(danse_engine* eng, int32_t on) {
  if (!eng) return fail(eng, "null engine");
  if (!eng->dxcpOn) return fail(eng, "DXCP-PhaT estimation is not on");
  HIPCHK(hipSetDevice(eng->dev));
  if (eng->graphExec) {   // the captured run changes
    (void)hipGraphExecDestroy(eng->graphExec);
    eng->graphExec = nullptr;
  }
  if (eng->dxRecFrames) (void)hipFree(eng->dxRecFrames);
  if (eng->dxRecOut) (void)hipFree(eng->dxRecOut);
  eng->dxRecFrames = nullptr;
  eng->dxRecOut = nullptr;
  eng->dxRecFeeds = 0;
  if (!on) return 0;
  const size_t P = (size_t)eng->S * (eng->k1 - eng->k0) * (eng->K - 1);
  const int feeds = eng->R / (kDxFrame / eng->Ns);
  if (feeds < 1) return 0;
  HIPCHK(dalloc(&eng->dxRecFrames, (size_t)feeds * P * 2 * kDxFrame));
  HIPCHK(dalloc(&eng->dxRecOut, (size_t)feeds * P * 2));
  HIPCHK(hipMemset(eng->dxRecFrames, 0, (size_t)feeds * P * 2 * kDxFrame * sizeof(float)));
  HIPCHK(hipMemset(eng->dxRecOut, 0, (size_t)feeds * P * 2 * sizeof(double)));
  eng->dxRecFeeds = feeds;
  return 0;
}

int danse_engine_dxcp_recorded(danse_engine* eng, int32_t* nFeeds, int32_t* nPairs, float* frames, size_t frameBytes,
                               double* out, size_t outBytes) {
  if (!eng || !nFeeds || !nPairs) return fail(eng, "null argument");
  const size_t P = (size_t)eng->S * (eng->k1 - eng->k0) * (eng->K - 1);
  *nFeeds = eng->dxRecFeeds;
  *nPairs = (int32_t)P;
  if (!eng->dxRecFrames) return 0;
  HIPCHK(hipSetDevice(eng->dev));
  HIPCHK(hipDeviceSynchronize());
  const size_t fb = (size_t)eng->dxRecFeeds * P * 2 * kDxFrame * sizeof(float);
  const size_t ob = (size_t)eng->dxRecFeeds * P * 2 * sizeof(double);
  if (frames) {
    if (frameBytes < fb) return fail(eng, "frame buffer too small");
    HIPCHK(hipMemcpy(frames, eng->dxRecFrames, fb, hipMemcpyDeviceToHost));
  }
  if (out) {
    if (outBytes < ob) return fail(eng, "output buffer too small");
    HIPCHK(hipMemcpy(out, eng->dxRecOut, ob, hipMemcpyDeviceToHost));
  }
  return 0;
}

int danse_engine_lanczos_stats(danse_engine* eng, int32_t* dst, size_t n) {
  if (!eng || !dst) return fail(eng, "null argument");
  if (n < (size_t)2 * eng->R) return fail(eng, "buffer too small: 2 R entries");
  HIPCHK(hipSetDevice(eng->dev));
  HIPCHK(hipDeviceSynchronize());
  if (!eng->lzStats) {
    std::fill(dst, dst + 2 * (size_t)eng->R, 0);
    return 0;
  }
  std::vector<int> h((size_t)2 * eng->R * kLzSlots);
  HIPCHK(hipMemcpy(h.data(), eng->lzStats, h.size() * sizeof(int), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < (size_t)2 * eng->R; ++i) {
    int acc = 0;
    for (int j = 0; j < kLzSlots; ++j) acc += h[i * kLzSlots + j];
    dst[i] = acc;
  }
  return 0;
}

int danse_mi355x_fill(void* ptr, int32_t value, size_t bytes, void* stream) {
  danse_engine* eng = nullptr;   // (HIPCHK's error slot)
  if (!ptr && bytes) return fail(eng, "null pointer");
  HIPCHK(fill_async(ptr, value, bytes, (hipStream_t)stream));
  return 0;
}

// node-sharded DXCP: the gathered z chunks of round r into the streams of
// the nodes this engine does not own (the received stream of every sender)
__global__ void zchunk_unpack_kernel(const float* __restrict__ zc, float* __restrict__ zStream, int S, int K, int k0,
                                     int k1, int Ns, int zLen, int r) {
  const long long n = (long long)S * K * Ns;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int i = (int)(e % Ns);
    const int s = (int)((e / Ns) % S);
    const int k = (int)(e / ((long long)Ns * S));
    if (k >= k0 && k < k1) continue;
    zStream[((long long)s * K + k) * zLen + (long long)r * Ns + i] = zc[e];
  }
}

int danse_engine_set_zchunk(danse_engine* eng, void* ptr) {
  if (!eng) return fail(eng, "null engine");
  if (eng->dFsTab) return fail(eng, "z-chunk exchange is for wholeChunk broadcasts");
  HIPCHK(hipSetDevice(eng->dev));
  eng->zChunk = (float*)ptr;
  if (eng->graphExec) {
    (void)hipGraphExecDestroy(eng->graphExec);
    eng->graphExec = nullptr;
    eng->graphR0 = eng->graphR1 = -1;
  }
  return 0;
}

int danse_engine_unpack_zchunk(danse_engine* eng, int32_t r, void* stream) {
  if (!eng || !eng->zChunk) return fail(eng, "no z-chunk buffer (danse_engine_set_zchunk)");
  if (r < 0 || r >= eng->R) return fail(eng, "round out of range");
  HIPCHK(hipSetDevice(eng->dev));
  const long long n = (long long)eng->S * eng->K * eng->Ns;
  hipLaunchKernelGGL(zchunk_unpack_kernel, dim3((unsigned)std::min<long long>((n + 255) / 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, eng->zChunk, eng->zStream, eng->S, eng->K, eng->k0, eng->k1, eng->Ns,
                     eng->zLen, r);
  HIPCHK(hipGetLastError());
  return 0;
}

int danse_engine_set_zspec(danse_engine* eng, void* ptr) {
  if (!eng || !ptr) return fail(eng, "null argument");
  HIPCHK(hipSetDevice(eng->dev));
  if (eng->ownZspec && eng->Zspec) HIPCHK(hipFree(eng->Zspec));
  eng->Zspec = (cf*)ptr;
  eng->ownZspec = false;
  if (eng->graphExec) {
    (void)hipGraphExecDestroy(eng->graphExec);
    eng->graphExec = nullptr;
    eng->graphR0 = eng->graphR1 = -1;
  }
  return 0;
}

int danse_engine_gate(danse_engine* eng, int32_t r, int32_t n, const int32_t* family, const int32_t* node,
                      const int32_t* scene, const double* qY, const double* qN, int32_t* verdict, void* stream) {
  if (!eng || !eng->y) return fail(eng, "inputs not set");
  if (r < 0 || r >= eng->R || n < 0) return fail(eng, "bad gate arguments");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(eng->dev));
  hipStream_t st = (hipStream_t)stream;
  std::vector<GateCand> h(n);
  int dmax = 1;
  for (int i = 0; i < n; ++i) {
    int fni = -1;
    for (size_t x = 0; x < eng->fns.size(); ++x)
      if (eng->fns[x].fam == family[i] && eng->fns[x].k == node[i]) fni = (int)x;
    if (fni < 0 || scene[i] < 0 || scene[i] >= eng->S) return fail(eng, "gate candidate not on this engine");
    h[i] = GateCand{fni, scene[i], qY[i], qN[i]};
    dmax = std::max(dmax, eng->fns[fni].D);
  }
  GateCand* dC = nullptr;
  int* dV = nullptr;
  HIPCHK(dalloc(&dC, (size_t)n));
  HIPCHK(dalloc(&dV, (size_t)n));
  std::vector<int> ones(n, 1);
  HIPCHK(hipMemcpyAsync(dC, h.data(), n * sizeof(GateCand), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(dV, ones.data(), n * sizeof(int), hipMemcpyHostToDevice, st));
  UpdateArgs a = make_update(eng, r);
  launch_gate(eng, a, dC, n, dmax, dV, st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(verdict, dV, n * sizeof(int), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  (void)hipFree(dC);
  (void)hipFree(dV);
  return 0;
}

int danse_engine_set_gate(danse_engine* eng, int32_t n, const int32_t* round, const int32_t* family,
                          const int32_t* node, const int32_t* scene, const double* qY, const double* qN) {
  if (!eng || n < 0) return fail(eng, "bad gate schedule");
  HIPCHK(hipSetDevice(eng->dev));
  if (eng->graphExec) {   // the captured run changes with the schedule
    (void)hipGraphExecDestroy(eng->graphExec);
    eng->graphExec = nullptr;
  }
  if (eng->dGateCand) (void)hipFree(eng->dGateCand);
  if (eng->dGateVerdict) (void)hipFree(eng->dGateVerdict);
  eng->dGateCand = nullptr;
  eng->dGateVerdict = nullptr;
  eng->nGate = 0;
  eng->gateOff.assign(eng->R + 1, 0);
  eng->gateDmax.assign(eng->R, 1);
  eng->gateHost.clear();
  if (n == 0) return 0;
  std::vector<std::pair<int, GateCand>> v;
  for (int i = 0; i < n; ++i) {
    int fni = -1;
    for (size_t x = 0; x < eng->fns.size(); ++x)
      if (eng->fns[x].fam == family[i] && eng->fns[x].k == node[i]) fni = (int)x;
    if (fni < 0 || scene[i] < 0 || scene[i] >= eng->S || round[i] < 0 || round[i] >= eng->R)
      return fail(eng, "gate candidate not on this engine");
    v.push_back({round[i], GateCand{fni, scene[i], qY[i], qN[i]}});
  }
  std::stable_sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  eng->gateHost = v;
  std::vector<GateCand> h;
  for (auto& x : v) {
    h.push_back(x.second);
    eng->gateOff[x.first + 1]++;
    eng->gateDmax[x.first] = std::max(eng->gateDmax[x.first], eng->fns[x.second.fni].D);
  }
  for (int r = 0; r < eng->R; ++r) eng->gateOff[r + 1] += eng->gateOff[r];
  eng->nGate = n;
  HIPCHK(dalloc(&eng->dGateCand, (size_t)n));
  HIPCHK(dalloc(&eng->dGateVerdict, (size_t)n));
  HIPCHK(hipMemcpy(eng->dGateCand, h.data(), n * sizeof(GateCand), hipMemcpyHostToDevice));
  return 0;
}

int danse_engine_gate_verdicts(danse_engine* eng, int32_t* verdict, void* stream) {
  if (!eng || !verdict) return fail(eng, "null argument");
  if (eng->nGate == 0) return 0;
  HIPCHK(hipSetDevice(eng->dev));
  HIPCHK(hipMemcpyAsync(verdict, eng->dGateVerdict, eng->nGate * sizeof(int), hipMemcpyDeviceToHost,
                        (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

int danse_engine_sro_estimates(danse_engine* eng, double* est, double* res) {
  if (!eng || !est || !res) return fail(eng, "null argument");
  const size_t n = (size_t)eng->S * eng->K * eng->R * (eng->K - 1);
  if (!eng->cohDrift && !eng->dxcpOn) {
    std::fill(est, est + n, 0.0);
    std::fill(res, res + n, 0.0);
    return 0;
  }
  HIPCHK(hipSetDevice(eng->dev));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(est, eng->cdEst, n * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(res, eng->cdRes, n * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

int danse_engine_set_flags(danse_engine* eng, const uint8_t* flags, void* stream) {
  if (!eng || !flags) return fail(eng, "null argument");
  HIPCHK(hipSetDevice(eng->dev));
  const size_t nb = (size_t)eng->R * eng->S * kMaxFam * eng->K;
  HIPCHK(hipMemcpyAsync(eng->dFlags, flags, nb, hipMemcpyHostToDevice, (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  if (eng->graphExec) {   // the split solves' launch sizes follow the flags
    (void)hipGraphExecDestroy(eng->graphExec);
    eng->graphExec = nullptr;
  }
  if (!eng->wideIds.empty()) build_wide_lists(eng, flags);
  return build_split_lists(eng, flags);
}

int danse_engine_zspec(danse_engine* eng, void** ptr, size_t* bytes) {
  if (!eng || !ptr || !bytes) return fail(eng, "null argument");
  *ptr = eng->Zspec;
  *bytes = (size_t)2 * eng->K * eng->S * eng->F * sizeof(cf);
  return 0;
}

// Resolve the device region of an output.  For per-family-node outputs the
// region is strided over scenes: (ptr, chunkBytes, sceneStrideBytes).
static int out_region(danse_engine* e, int which, int family, int node, char** ptr, size_t* chunk, size_t* stride,
                      int* nChunks) {
  const int S = e->S, K = e->K, F = e->F;
  *nChunks = S;
  if (which == DANSE_OUT_W || which == DANSE_OUT_WEXT) {
    if (node < e->k0 || node >= e->k1) return fail(e, "node not owned by this engine");
    const long long hw = e->keepHistory ? (long long)e->R + 1 : 2;
    if (which == DANSE_OUT_W) {
      const FamNode* fn = nullptr;
      for (auto& x : e->fns)
        if (x.fam == family && x.k == node) fn = &x;
      if (!fn) return fail(e, "family not computed");
      *ptr = (char*)(e->wHist + fn->wOff);
      *chunk = (size_t)hw * F * fn->D * sizeof(cf);
      *stride = (size_t)e->wStride * sizeof(cf);
    } else {
      *ptr = (char*)(e->wExtHist + e->wExtNodeOff[node]);
      *chunk = (size_t)hw * F * e->M[node] * sizeof(cf);
      *stride = (size_t)e->wExtStride * sizeof(cf);
    }
    return 0;
  }
  *nChunks = 1;
  *stride = 0;
  if (which == DANSE_OUT_D) {
    if (!((e->families >> family) & 1)) return fail(e, "family not computed");
    *ptr = (char*)(e->d + (long long)family * S * K * e->T);
    *chunk = (size_t)S * K * e->T * sizeof(float);
  } else if (which == DANSE_OUT_DHAT) {
    if (!((e->families >> family) & 1)) return fail(e, "family not computed");
    *ptr = (char*)(e->dhat + (long long)family * S * K * e->R * F);
    *chunk = (size_t)S * K * e->R * F * sizeof(cf);
  } else if (which == DANSE_OUT_Z) {
    *ptr = (char*)e->zStream;
    *chunk = (size_t)S * K * e->zLen * sizeof(float);
  } else if (which == DANSE_OUT_DIAG) {
    *ptr = (char*)e->diag;
    *chunk = (size_t)S * K * kMaxFam * sizeof(int);
  } else {
    return fail(e, "unknown output");
  }
  return 0;
}

int danse_engine_put(danse_engine* eng, int32_t which, int32_t family, int32_t node, const void* src, size_t bytes,
                     void* stream) {
  if (which != DANSE_OUT_W && which != DANSE_OUT_WEXT) return fail(eng, "only W / WEXT can be loaded");
  char* p;
  size_t chunk, stride;
  int n;
  int rc = out_region(eng, which, family, node, &p, &chunk, &stride, &n);
  if (rc) return rc;
  if (bytes < chunk * n) return fail(eng, "source too small");
  HIPCHK(hipSetDevice(eng->dev));
  HIPCHK(hipMemcpy2DAsync(p, stride, src, chunk, chunk, n, hipMemcpyDefault, (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

int danse_engine_output_bytes(danse_engine* eng, int32_t which, int32_t family, int32_t node, size_t* bytes) {
  char* p;
  size_t chunk, stride;
  int n;
  int rc = out_region(eng, which, family, node, &p, &chunk, &stride, &n);
  if (rc) return rc;
  *bytes = chunk * n;
  return 0;
}

int danse_engine_get(danse_engine* eng, int32_t which, int32_t family, int32_t node, void* dst, size_t bytes,
                     void* stream) {
  char* p;
  size_t chunk, stride;
  int n;
  int rc = out_region(eng, which, family, node, &p, &chunk, &stride, &n);
  if (rc) return rc;
  if (bytes < chunk * n) return fail(eng, "destination too small");
  HIPCHK(hipSetDevice(eng->dev));
  if (n == 1) {
    HIPCHK(hipMemcpyAsync(dst, p, chunk, hipMemcpyDefault, (hipStream_t)stream));
  } else {
    HIPCHK(hipMemcpy2DAsync(dst, chunk, p, stride, chunk, n, hipMemcpyDefault, (hipStream_t)stream));
  }
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}


// ---------------------------------------------------------------------------
// Fine-grained operators
// ---------------------------------------------------------------------------

__global__ void __launch_bounds__(256) wola_analysis_kernel(const float* x, int T, const int* ends, const float* win,
                                                            int N, int Ns, cf* out, const cf* tw) {
  __shared__ cf b0[1024];
  __shared__ cf b1[1024];
  const int c = blockIdx.x;
  load_frame(b0, x + (long long)c * T, ends[c], N, T, win);
  __syncthreads();
  cf* o = fft1024(b0, b1, tw);
  const float inv = 1.0f / sqrtf((float)Ns);
  const int F = N / 2 + 1;
  for (int f = threadIdx.x; f < F; f += blockDim.x) out[(long long)c * F + f] = inv * o[f];
}

int danse_wola_analysis(const float* x, int32_t C, int32_t T, const int32_t* ends, const float* win, int32_t N,
                        int32_t Ns, float* out, void* stream) {
  danse_engine* eng = nullptr;
  if (N != 1024) return fail(nullptr, "only N = 1024");
  static cf* tw = nullptr;
  if (!tw) {
    std::vector<cf> h(N);
    for (int m = 0; m < N; ++m) {
      const double ang = -2.0 * M_PI * m / N;
      h[m] = cf{(float)std::cos(ang), (float)std::sin(ang)};
    }
    HIPCHK(dalloc(&tw, N));
    HIPCHK(hipMemcpy(tw, h.data(), N * sizeof(cf), hipMemcpyHostToDevice));
  }
  hipLaunchKernelGGL(wola_analysis_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream, x, T, ends, win, N, Ns,
                     (cf*)out, tw);
  HIPCHK(hipGetLastError());
  return 0;
}

int danse_filter_update(const double* Ryy, const double* Rnn, int32_t B, int32_t D, int32_t gevd, int32_t rank,
                        int32_t ref, float* w, int32_t* diag, void* stream) {
  danse_engine* eng = nullptr;
  if (D < 1 || D > wide::kMaxD) return fail(nullptr, "D must be in [1, 256]");
  if (gevd && (rank < 1 || rank > kRMax || rank > D)) return fail(nullptr, "bad rank");
  if (ref < 0 || ref >= D) return fail(nullptr, "bad reference index");
  if (D > kMaxDMax) {
    // wide class (wide.hpp): one workgroup per bin, float64 workspace
    // (stream-ordered, released behind the launches)
    hipStream_t st = (hipStream_t)stream;
    wide::WideArgs wa{};
    wa.D = D; wa.rank = rank; wa.gevd = gevd; wa.F = 1; wa.nItems = B; wa.layout = 0;
    wa.RyyD = (const cd*)Ryy; wa.Rnn = (const cd*)Rnn; wa.srcScene = (long long)D * D; wa.srcBin = 0;
    wa.nOut = 1; wa.refs[0] = ref; wa.wOff[0] = 0; wa.w = (cf*)w; wa.wScene = D; wa.wBin = 0;
    wa.diag = diag;
    const long long chunk = wide::chunk_for(D, B);
    HIPCHK(hipMallocAsync((void**)&wa.work, (size_t)chunk * wide::work_elems(D) * sizeof(cd), st));
    const hipError_t le = wide::launch_wide_filters(wa, chunk, st);
    const hipError_t fe = hipFreeAsync(wa.work, st);   // (released on the error path too)
    HIPCHK(le);
    HIPCHK(fe);
    return 0;
  }
  int G, DM;
  pick_class(D, G, DM);
  hipStream_t st = (hipStream_t)stream;
  const cd* a = (const cd*)Ryy;
  const cd* n = (const cd*)Rnn;
  cf* o = (cf*)w;
  launch_filter_update_class(DM, a, n, B, D, gevd, rank, ref, o, diag, st);
  HIPCHK(hipGetLastError());
  return 0;
}
