// Device kernels of the DANSE frame-update engine.
//
// Per DANSE round r (all nodes of all scenes in parallel; round-synchronous
// fully connected schedule):
//   bcast_kernel  (one 256-thread workgroup per (scene, node)):
//       [synthesis of the estimates of round r-1 (get_desired_sig_chunk,
//        d_base.py:2027-2084)]
//       WOLA analysis of the broadcast frame of every local mic
//        (d_base.py:1821-1826), fused-signal spectrum zhat = wExt^H yhat,
//       WOLA synthesis + OLA normalisation of z (d_base.py:1829-1852),
//       append z[:Ns] to the node's stream (fill_buffers, d_classes.py:1185),
//       analysis of the z frame every receiver will use
//        (process_incoming_signals_buffers + build_ytilde,
//         d_classes.py:1701-1807,1893-1934).
//   update kernels (kernels_lane.hpp: one bin per lane, D <= 12;
//       kernels_big.hpp: one bin per wavefront, D <= 64):
//       SCM update (d_classes.py:2048-2267), filter update (update_w /
//       update_w_gevd, d_classes.py:3320-3387), external filters
//       (d_classes.py:1627-1694), dhat = w^H yhat (d_base.py:2075).
#pragma once
#include "common.hpp"
#include "solver.hpp"
#include "../../include/danse_mi355x_defs.h"

namespace danse {

constexpr int kMaxFam = 4;

struct FamNode {
  int fam, k, D, ref;
  int chanOff;        // offset into chanList
  int extMode;        // DANSE family only (else -1)
  int M;              // local mics of node k
  int packed;         // SCM layout (scm_lower): 1 packed lower triangles bin-minor [D(D+1)/2][F] (lane
                      // classes), 2 packed lower triangles bin-major [F][D(D+1)/2] (D > 12), 0 rows
                      // [F][D][D] (the D <= 12 grid classes of smallDGrid / the resident engine)
  long long scmOff;   // complex-element offset within one scene's SCM block
  long long wOff;     // complex-element offset within one scene's w-history block
  long long wExtOff;  // DANSE only: offset within one scene's wExt-history block
  long long tgtOff;   // DANSE only: offset within one scene's target block
  long long liOff;    // lane classes, GEVD: offset of the factor cache (Li, g) within one scene's block
  long long vOff;     // lane-grid classes, GEVD: offset of the eigenvector cache (solver2d.hpp lanczos2d), -1 none
  long long l64Off;   // lane-grid classes, GEVD: offset of the float64 factor record (solver2d.hpp li_rank1_2d), -1 none
  long long cOff;     // one-bin-per-wave grid classes, GEVD: offset of the C = Li Ryy Li^H cache (kernels_2d.hpp), -1 none
};

struct UpdateArgs {
  int S, K, MT, F, R, r;
  int nFN;                 // family-nodes in this launch
  const FamNode* fn;       // [nFN]
  const int* famNodeId;    // [nFN] index into the global family-node list (for flags/dhat)
  const int* chanList;
  const uint8_t* flags;    // [R][S][kMaxFam][K]
  const cf* Yspec;         // [2][S][MT][F]
  const cf* Zspec;         // [2][K][S][F]: slot r & 1 holds the senders' round-r frames
  const uint8_t* zLag;     // [R][K][K] or null: 1 = consume sender q's round r-1 frame (SROs)
  const double* zPhase;    // [R][K][K] or null: SRO phase-compensation offsets (samples)
  cf* Ryy;                 // per scene stride scmStride (complex float)
  cd* Rnn;                 // same element offsets, complex double (DESIGN.md "Precision")
  long long scmStride;
  cf* wHist;               // per scene stride wStride
  long long wStride;
  int wHistory;            // 1: [R+1][F][D] per family-node; 0: 2 slots
  cf* wExtHist;
  long long wExtStride;
  int wExtHistory;
  cf* wExtTarget;
  long long tgtStride;
  cf* dhat;                // [fam][S][K][R][F]
  const double* beta;      // [S*K]
  const float* betaExt;    // [S*K]
  float alphaExt;
  int gevd, rank;
  int* diag;               // [S*K*kMaxFam]
  cf* liCache;             // GEVD factor cache per family-node [NT + D][F] (Li = L^-1 packed, g = L^H e_ref)
  cf* liLane;              // lane classes: the same records in wave order, [block][entry][64] (kernels_lane.hpp)
  const double* cdPhase;   // CohDrift phase accumulator [S][K][K] (adds to zPhase), or null
  long long liStride;      // per scene; null cache = always refactor
  // centralised / SSBC under asynchronous clocks (danse_cfg.cEnd): channel
  // codes >= MT + K name raw channel (code - MT - K) of another node, read
  // from Cspec [2][S][MT][F] (slot r & 1 holds the senders' round-r raw
  // frames) with that sender's zLag
  const cf* Cspec;
  const int* chanNode;     // [MT] node of each channel
  const double* cPhase;    // [R][K][MT] centralised compensation phase (samples), or null
  // resident engine (resident.hpp): the update-frame spectra of every round
  // ([R][S][MT][F], replacing the Yspec ping-pong) and the fused spectra of
  // every round (Zspec = [R + 1][K][S][F], slot r + 1 = round r, slot 0
  // zeros), read with agent-coherent loads (written inside the same launch)
  const cf* Yall;
  int zAll;
  // lane classes, split solves (kernels_2d.hpp PK): the lane kernel skips the
  // (scene, family-node) items that solve this round; the packed-storage
  // lane-grid kernel runs them, one launch item per entry of solveItems
  int splitSolve;
  const int* solveItems;   // this round's solving items (s * nFN + fni)
  // no item of this launch's class solves this round (host, from the flag
  // table): the recursion-only kernel variants run, not held to the solver's
  // registers / LDS
  int noSolve;
  // pre-solve prefix fast-forward (span.hpp): this round's SCM recursion is
  // deferred to span_rec_kernel; the recursion-only variants run their tail
  // (filters, external filters, d-hat) only
  int noRec;
  // fewSamples step lists (compile_rounds_fs): the nodes this launch updates
  // (bit k: node k); the others are left untouched
  unsigned nodeMask;
  // lane-grid GEVD classes: per bin the eigenvector of C of the previous
  // solve ([F][DMAX] per family-node at FamNode.vOff, per scene stride
  // vStride), the warm start of the rank-1 Lanczos path; null = off
  cf* vCache;
  long long vStride;
  // lane-grid GEVD classes: per bin the float64 factor of the last
  // factorisation (Li packed + row ref of L, [F][l64_record] per family-node
  // at FamNode.l64Off, per scene stride l64Stride): a solve one noise frame
  // after it updates it by rank one instead of refactoring; null = off
  cd* l64Cache;
  long long l64Stride;
  // [R][2][kLzSlots] or null: per round the bins whose warm Lanczos solve was
  // accepted and those sent back to the Householder path (diagnostics; the
  // host sums the slots)
  int* lzStats;
  // one-bin-per-wave lane-grid GEVD classes: per bin C = Li Ryy Li^H of the
  // last solve in the lane-grid block layout ([F][NB * NB][64] per
  // family-node at FamNode.cOff, per scene stride cStride): a solve on the
  // cached factor updates it by rank one (c_reusable) instead of the O(D^3)
  // congruence; null = off
  cf* cCache;
  long long cStride;
  // the solves on the cached factor and C run on update_kernel_2dc this round
  // (items listed in creItems, their failed warm solves in fbList / fbCount
  // for fallback_kernel_2d): update_kernel_2d skips them
  int leanOn;              // VAD-frame solves on update_kernel_2dc<NB, false>
  int leanNoise;           // noise-frame solves on update_kernel_2dc<NB, true>
  const int* creItems;     // this round's items (s * nFN + fni) for update_kernel_2dc<NB, false>
  const int* cnItems;      // this round's items for update_kernel_2dc<NB, true>
  int* fbList;             // failed warm solves (item * F + f)
  int* fbCount;            // their count (one counter per round)
  // DANSE_STAMP builds only (diagnostics): per launch wave, kStampN shader
  // clock marks + a path code (update_kernel_2d), or null
  unsigned long long* stamps;
};

constexpr int kLzSlots = 64;
constexpr int kStampN = 9;   // marks per wave; slot kStampN holds the path code
#ifndef DANSE_STAMP
#define DANSE_STAMP 0   // diagnostics build (danse_amd.build variant 'stamp'): per-wave phase clocks
#endif

DANSE_DEV bool node_in(unsigned mask, int k) { return ((mask >> k) & 1u) != 0u; }

// Element (i, j), i >= j, of scene s's bin-f SCM of a family-node, in the
// family-node's layout (FamNode.packed).  In the packed layouts only the lower
// triangle exists: (j, i) is conj((i, j)), the diagonal is real.
DANSE_DEV long long scm_lower(const FamNode& d, long long scmStride, int s, int F, int f, int i, int j) {
  const long long b = (long long)s * scmStride + d.scmOff;
  const int t = i * (i + 1) / 2 + j;
  if (d.packed == 1) return b + (long long)t * F + f;
  if (d.packed == 2) return b + (long long)f * (d.D * (d.D + 1) / 2) + t;
  return b + ((long long)f * d.D + i) * d.D + j;
}

// The wide family-nodes (D > kMaxDMax, the online centralised family above 64
// channels) keep Ryy in float64 as Rnn, in the Rnn array F T entries past
// their Rnn (scmOff reserves both): the reference's float64 SCMs, which the
// start gate's rank / PSD test at sum(M) = 256 needs (a 256 x 256 Ryy after
// 257 averaged frames is nearly singular; its float32 rounding fails the
// check rounds after the float64 matrix passes it)
DANSE_DEV bool wide_fn(const FamNode& d) { return d.D > 64; }
DANSE_DEV long long wide_ryy_shift(const FamNode& d, int F) { return (long long)F * (d.D * (d.D + 1) / 2); }
// an SCM entry as the gate reads it (Ryy: complex64, or the wide fns' float64)
DANSE_DEV cd scm_entry(const UpdateArgs& a, const FamNode& d, bool ryy, long long ee) {
  if (!ryy) return a.Rnn[ee];
  return wide_fn(d) ? a.Rnn[ee + wide_ryy_shift(d, a.F)] : cdk(a.Ryy[ee]);
}

// Agent-coherent (sc1) 8-byte load / store of a complex value: the resident
// engine's hand-offs between waves of one launch (payload stored sc1 and
// loaded sc1, flag after s_waitcnt vmcnt(0): MI355X_MICROARCH.md,
// inter-workgroup visibility, first hand-off row).  Global address space so
// that they lower to global_load / global_store (never flat).
typedef __attribute__((address_space(1))) unsigned long long danse_gu64;
typedef __attribute__((address_space(1))) unsigned int danse_gu32;
DANSE_DEV cf ld_sc1(const cf* p) {
  const unsigned long long v =
      __hip_atomic_load((danse_gu64*)(const_cast<cf*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return cf{__uint_as_float((unsigned)(v & 0xffffffffull)), __uint_as_float((unsigned)(v >> 32))};
}
DANSE_DEV void st_sc1(cf* p, cf x) {
  const unsigned long long v = (unsigned long long)__float_as_uint(x.re) | ((unsigned long long)__float_as_uint(x.im) << 32);
  __hip_atomic_store((danse_gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DANSE_DEV unsigned ld_flag(const unsigned* p) {
  return __hip_atomic_load((danse_gu32*)(const_cast<unsigned*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DANSE_DEV void st_flag(unsigned* p, unsigned v) {
  __hip_atomic_store((danse_gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// yhat *= exp(-j 2 pi f phi / N) (compensate_sros, d_classes.py:1936-2046)
DANSE_DEV cf sro_rotate(cf v, int f, int F, double ph) {
  double t = (double)f * ph / (double)(2 * (F - 1));
  t -= rint(t);
  float sn, cs;
  sincospif(-2.0f * (float)t, &sn, &cs);
  return v * cf{cs, sn};
}

// The factor of Rnn cached by the last solve of this (scene, family-node) is
// still the factor of the current Rnn: no Rnn update since that solve (the
// flags of the rounds in between; Rnn changes only on VAD-inactive frames,
// and the cached factor was taken after that round's own update).
// Wave-uniform scan over at most kLiScan earlier rounds of the flag table.
constexpr int kLiScan = 64;
DANSE_DEV bool li_reusable(const UpdateArgs& a, const FamNode& d, int s, int opN) {
  if (!a.liCache || opN != DANSE_OP_KEEP) return false;
  for (int rr = a.r - 1; rr >= 0 && rr >= a.r - kLiScan; --rr) {
    const uint8_t f2 = a.flags[(((long long)rr * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
    if ((f2 & DANSE_FLAG_SOLVE) && !(f2 & DANSE_FLAG_PREGIVEN)) return true;
    if (((f2 >> 2) & 3) != DANSE_OP_KEEP) return false;
  }
  return false;
}

// li_reusable with the flags of round r - 1 already loaded (flPrev; the
// caller's own flags when r = 0, which the r > 0 test ignores)
DANSE_DEV bool li_reusable_prev(const UpdateArgs& a, const FamNode& d, int s, int opN, uint8_t flPrev) {
  if (!a.liCache || opN != DANSE_OP_KEEP || a.r == 0) return false;
  if ((flPrev & DANSE_FLAG_SOLVE) && !(flPrev & DANSE_FLAG_PREGIVEN)) return true;
  if (((flPrev >> 2) & 3) != DANSE_OP_KEEP) return false;
  for (int rr = a.r - 2; rr >= 0 && rr >= a.r - kLiScan; --rr) {
    const uint8_t f2 = a.flags[(((long long)rr * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
    if ((f2 & DANSE_FLAG_SOLVE) && !(f2 & DANSE_FLAG_PREGIVEN)) return true;
    if (((f2 >> 2) & 3) != DANSE_OP_KEEP) return false;
  }
  return false;
}

// The float64 factor record of the last solve is the factor of Rnn before
// this round's single rank-one update (opN == AVG; every round since that
// solve left Rnn alone): solver2d.hpp li_rank1_2d moves it to this round's.
DANSE_DEV bool li_updatable(const UpdateArgs& a, const FamNode& d, int s, int opN) {
  if (!a.l64Cache || d.l64Off < 0 || opN != DANSE_OP_AVG) return false;
  for (int rr = a.r - 1; rr >= 0 && rr >= a.r - kLiScan; --rr) {
    const uint8_t f2 = a.flags[(((long long)rr * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
    if ((f2 & DANSE_FLAG_SOLVE) && !(f2 & DANSE_FLAG_PREGIVEN)) return true;
    if (((f2 >> 2) & 3) != DANSE_OP_KEEP) return false;
  }
  return false;
}

// The C = Li Ryy Li^H cached by the last solve of this family-node is C of
// the current factor and of Ryy before this round's update: the factor is
// reused (li_reusable) and no round since that solve updated either SCM.
// This round's Ryy update then moves C by the same rank one, through Li y.
// (every kCRefresh-th round, r % kCRefresh == 0, takes the full congruence
// instead: the rank-one moves of the cached C, exact in arithmetic, carry
// float32 roundings from frame to frame, the noise-frame transforms without
// the forgetting factor's decay.  Whole rounds, not a stagger over items: a
// partial full-kernel launch every round cost N2 10 ms per run)
constexpr int kCRefresh = 32;
DANSE_DEV bool c_reusable(const UpdateArgs& a, const FamNode& d, int s) {
  for (int rr = a.r - 1; rr >= 0 && rr >= a.r - kLiScan; --rr) {
    const uint8_t f2 = a.flags[(((long long)rr * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
    if ((f2 & DANSE_FLAG_SOLVE) && !(f2 & DANSE_FLAG_PREGIVEN)) return true;
    if ((f2 & 15) != 0) return false;   // (opY | opN << 2: an SCM update without a solve)
  }
  return false;
}

// Observation vector entry of lane li (channel chanList[chanOff + li]) for
// bin f: a local spectrum, or the fused spectrum of sender q (the frame of
// round r or r-1, zLag) with the SRO phase compensation
// yhat *= exp(-j 2 pi f phi / N) of compensate_sros (d_classes.py:1936-2046).
DANSE_DEV cf load_y_c(const UpdateArgs& a, const FamNode& d, int s, int f, int c, bool act);
DANSE_DEV int chan_of(const UpdateArgs& a, const FamNode& d, int li, bool act) {
  return a.chanList[d.chanOff + (act ? li : 0)];
}
DANSE_DEV cf load_y(const UpdateArgs& a, const FamNode& d, int s, int f, int li, bool act) {
  return load_y_c(a, d, s, f, chan_of(a, d, li, act), act);
}
// (the same, from the channel id: callers that issue other loads between the
// channel-id load and the spectrum load)
DANSE_DEV cf load_y_c(const UpdateArgs& a, const FamNode& d, int s, int f, int c, bool act) {
  const int F = a.F, r = a.r;
  const int rawBase = a.MT + a.K;
  cf v;
  if (c < a.MT) {
    v = a.Yall ? a.Yall[(((long long)r * a.S + s) * a.MT + c) * F + f]
               : a.Yspec[(((long long)((r + 1) & 1) * a.S + s) * a.MT + c) * F + f];
  } else if (c >= rawBase) {
    // another node's raw channel in the centralised / SSBC vector
    // (process_incoming_signals_buffers_centr, d_classes.py:1809-1891)
    const int ch = c - rawBase;
    const int q = a.chanNode[ch];
    const int lag = a.zLag ? a.zLag[((long long)r * a.K + d.k) * a.K + q] : 0;
    v = a.Cspec[(((long long)((r - lag) & 1) * a.S + s) * a.MT + ch) * F + f];
  } else {
    const int q = c - a.MT;
    const long long lk = ((long long)r * a.K + d.k) * a.K + q;
    const int lag = a.zLag ? a.zLag[lk] : 0;
    if (a.zAll) v = ld_sc1(a.Zspec + ((((long long)(r - lag + 1)) * a.K + q) * a.S + s) * F + f);
    else v = a.Zspec[((((long long)((r - lag) & 1)) * a.K + q) * a.S + s) * F + f];
    if (a.zPhase) {
      double ph = a.zPhase[lk];
      if (a.cdPhase) ph += a.cdPhase[((long long)s * a.K + d.k) * a.K + q];
      v = sro_rotate(v, f, F, ph);
    }
  }
  if (a.cPhase && d.fam == DANSE_FAM_CENTR) {
    // phaseShiftFactorsCentr of every channel of the centralised vector
    // (d_classes.py:1996-2038), own channels included
    const int ch = (c < a.MT) ? c : c - rawBase;
    v = sro_rotate(v, f, F, a.cPhase[((long long)r * a.K + d.k) * a.MT + ch]);
  }
  return csel(act, v, cf{0.0f, 0.0f});
}

// load_y of entries 0..D-1 (all active) of one lane, for the lane kernels:
// the same values and arithmetic, the loads issued stage by stage over all
// entries -- channel ids; sender node, lag and phases; the spectra -- so that
// each stage is one memory round trip (hold()) instead of a dependent chain
// per entry under per-entry branches.  Indices of the loads an entry does not
// need are clamped to valid ones and their values discarded.
// (nAct: the entries past it repeat entry nAct - 1 -- a caller compiled for a
// larger size than the family-node's D)
template <int D>
DANSE_DEV void load_y_all(const UpdateArgs& a, const FamNode& d, int s, int f, cf (&y)[D], int nAct = D) {
  const int F = a.F, r = a.r, K = a.K, MT = a.MT;
  const int rawBase = MT + K;
  int c[D];
#pragma unroll
  for (int i = 0; i < D; ++i) c[i] = a.chanList[d.chanOff + min(i, nAct - 1)];
  hold(c);
  // sender node q (fused spectra) / raw channel's node (centralised vector)
  int q[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    const bool raw = c[i] >= rawBase;
    q[i] = (c[i] >= MT && !raw) ? c[i] - MT : 0;
    if (a.chanNode) {
      const int nq = a.chanNode[raw ? c[i] - rawBase : 0];
      q[i] = raw ? nq : q[i];
    }
  }
  if (a.chanNode) hold(q);
  const long long lk0 = ((long long)r * K + d.k) * K;
  // (the optional tables tested once, outside the unrolled loops: a test
  // per element is a branch per element, and a wait inside each)
  int lag[D];
  double ph[D], cph[D];
#pragma unroll
  for (int i = 0; i < D; ++i) lag[i] = 0, ph[i] = 0.0, cph[i] = 0.0;
  // (each table's loads issued before the previous table's are waited for)
  if (a.zLag) {
#pragma unroll
    for (int i = 0; i < D; ++i) lag[i] = a.zLag[lk0 + q[i]];
  }
  if (a.zPhase) {
#pragma unroll
    for (int i = 0; i < D; ++i) ph[i] = a.zPhase[lk0 + q[i]];
  }
  if (a.cPhase) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const int ch = (c[i] < MT) ? c[i] : (c[i] >= rawBase ? c[i] - rawBase : 0);
      cph[i] = a.cPhase[((long long)r * K + d.k) * MT + ch];
    }
  }
  if (a.zLag) hold(lag);
  if (a.zPhase) hold(ph);
  if (a.cPhase) hold(cph);
  if (a.cdPhase) {
#pragma unroll
    for (int i = 0; i < D; ++i) ph[i] += a.cdPhase[((long long)s * K + d.k) * K + q[i]];
  }
  const cf* pv[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    const bool loc = c[i] < MT, raw = c[i] >= rawBase;
    const cf* p;
    if (loc) {
      p = a.Yall ? a.Yall + (((long long)r * a.S + s) * MT + c[i]) * F + f
                 : a.Yspec + (((long long)((r + 1) & 1) * a.S + s) * MT + c[i]) * F + f;
    } else if (raw) {
      p = a.Cspec + (((long long)((r - lag[i]) & 1) * a.S + s) * MT + (c[i] - rawBase)) * F + f;
    } else {
      p = a.zAll ? a.Zspec + ((((long long)(r - lag[i] + 1)) * K + q[i]) * a.S + s) * F + f
                 : a.Zspec + ((((long long)((r - lag[i]) & 1)) * K + q[i]) * a.S + s) * F + f;
    }
    pv[i] = p;
  }
  // (the load kind tested once: a select per element between the plain and
  // the sc1 load was a branch per element, each load waited for in its own)
  cf v[D];
  if (a.zAll) {
#pragma unroll
    for (int i = 0; i < D; ++i) v[i] = ld_sc1(pv[i]);
    hold(v);
  } else {
#pragma unroll
    for (int i = 0; i < D; ++i) v[i] = *pv[i];
    hold(v);
  }
#pragma unroll
  for (int i = 0; i < D; ++i) {
    const bool loc = c[i] < MT, raw = c[i] >= rawBase;
    cf x = v[i];
    if (!loc && !raw && a.zPhase) x = sro_rotate(x, f, F, ph[i]);
    if (a.cPhase && d.fam == DANSE_FAM_CENTR) x = sro_rotate(x, f, F, cph[i]);
    y[i] = x;
  }
}

// Relaxed external filter entry b wExt[i] + (1 - b) target (one function
// for every caller, so that every caller rounds it alike)
DANSE_DEV cf ext_relax(float be, cf ep, cf tg) { return be * ep + (1.0f - be) * tg; }

// External filters (DANSE family, update_external_filters,
// d_classes.py:1627-1694) and dhat = w^H yhat (d_base.py:2075, DC / Nyquist
// forced real, quirk Q7) of one (scene, family-node, bin); lane li of the
// bin's lane group holds w_li, dh is the group sum of conj(w) y.  Returns
// the new external filter entry li (DANSE family, li < M; else zero).
DANSE_DEV cf node_bin_tail(const UpdateArgs& a, const FamNode& d, int s, int f, int li, uint8_t fl, bool pregiven,
                             bool valid, cf w, cf y, cf dh) {
  const int F = a.F;
  const int r = a.r;
  cf ne = cf{0.0f, 0.0f};
  if (d.extMode >= 0 && !pregiven) {
    const int M = d.M;
    const long long eb = (long long)s * a.wExtStride + d.wExtOff;
    const int eP = a.wExtHistory ? r : (r & 1);
    const int eN = a.wExtHistory ? r + 1 : ((r + 1) & 1);
    cf* eprev = a.wExtHist + eb + ((long long)eP * F + f) * M;
    cf* enext = a.wExtHist + eb + ((long long)eN * F + f) * M;
    cf* tgt = a.wExtTarget + (long long)s * a.tgtStride + d.tgtOff + (long long)f * M;
    if (li < M && valid) {
      if (d.extMode == 0) ne = w;
      else if (d.extMode == 2) ne = eprev[li];
      else if (d.extMode == 3) ne = cf{(li == d.ref) ? 1.0f : 0.0f, 0.0f};
      else {
        const float be = a.betaExt[s * a.K + d.k];
        const cf tg = tgt[li];
        ne = ext_relax(be, eprev[li], tg);
        if (fl & DANSE_FLAG_EXT_TARGET) tgt[li] = (1.0f - a.alphaExt) * tg + a.alphaExt * w;
      }
      enext[li] = ne;
    }
  }
  if (f == 0 || f == F - 1) dh.im = 0.0f;
  if (li == 0 && valid) {
    a.dhat[((((long long)d.fam * a.S + s) * a.K + d.k) * a.R + r) * F + f] = dh;
  }
  return ne;
}

}  // namespace danse
