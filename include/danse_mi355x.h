/*
 * danse_mi355x.h — C-ABI of the MI355X DANSE frame-update engine.
 *
 * Drop-in boundary for the reference's swappable unit
 *   danse_function(wasnObj, p) -> (dv, wasnObj)      tests/sandbox.py:112-129,
 *                                                      danse_toolbox/d_core.py:26-102
 * whose per-event operators are
 *   dv.broadcast(t, fs, k)                            danse_toolbox/d_classes.py:1043-1128
 *   dv.update_and_estimate(t, fs, k, bypass)          danse_toolbox/d_classes.py:1252-1330
 * and whose batch counterparts are
 *   batch_update_danse_covmats / perform_update / batch_estimate
 *                                                      danse_toolbox/d_batch.py:127-152
 *
 * The reference has no FFI (it is pure Python); the binding a maintainer adds
 * is the ctypes stub in INTEGRATION.md.  Conventions:
 *   - plain pointers and sizes only; complex numbers are interleaved float32
 *     {re, im}; device pointers are hipMalloc'd (or torch) GPU memory;
 *   - the engine owns all of its device state; inputs are borrowed for the
 *     duration of the call that receives them;
 *   - every entry point returns 0 on success and a negative code on error;
 *     danse_last_error() returns the message; no exception crosses the ABI;
 *   - one engine per device/stream; not internally thread-safe.
 */
#ifndef DANSE_MI355X_H
#define DANSE_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#include "danse_mi355x_defs.h"

typedef struct danse_cfg {
  /* sizes */
  int32_t S;            /* independent scenes (same shape) batched in one engine */
  int32_t K;            /* nodes per scene (fully connected)                      */
  const int32_t* M;     /* [K] sensors per node                                   */
  int32_t N;            /* DFT size (DFTsize)                                     */
  int32_t Ns;           /* hop (N * (1 - WOLAovlp))                               */
  int32_t T;            /* samples per channel                                    */
  int32_t R;            /* rounds (DANSE iterations) to run                       */
  int32_t k0, k1;       /* nodes owned by this engine (multi-GPU sharding), [k0,k1) */
  /* algorithm */
  int32_t gevd;         /* performGEVD                                            */
  int32_t rank;         /* GEVDrank                                               */
  int32_t ref;          /* referenceSensor                                        */
  int32_t families;     /* bitmask of enum danse_family                           */
  float alphaExt;       /* alphaExternalFilters                                   */
  const int32_t* extMode;   /* [K]                                                */
  const double* beta;       /* [S*K] SCM forgetting factor per (scene, node)      */
  const float* betaExt;     /* [S*K] external-filter forgetting factor            */
  const float* winAnalysis; /* [N] */
  const float* winSynthesis;/* [N] */
  /* schedule (host-computed from the reference event matrix, d_base.py:513-1225) */
  const int32_t* bcEnd;     /* [R*K] broadcast frame end sample  floor(t fs)       */
  const int32_t* upEnd;     /* [R*K] update frame end  floor(t fs) - (N - Ns)      */
  const uint8_t* flags;     /* [R*S*DANSE_MAX_FAMILIES*K] control bytes (above)    */
  /* initial state, host memory (copied at create) */
  const float* w0;          /* initial filters, per family f, node k (all K nodes,
                               family-major): [F][D_fk] complex, same for every
                               scene; NULL = zeros                                 */
  const float* wExt0;       /* initial external filters, per node: [F][M_k] complex */
  const float* wExtTarget0; /* initial external-filter targets, same layout        */
  const double* scmInit;    /* initial SCM slice per family-node: [D][D] complex
                               double, tiled over bins and scenes (Ryy = Rnn;
                               Rnn is kept in double, Ryy in float); NULL = 0     */
  int32_t keepHistory;      /* 1: keep w / wExt for every iteration (reference
                               layout needs it for the SNR replay)                  */
  /* asynchronous clocks (SROs), host-computed from the event order
   * (fill_buffers / process_incoming_signals_buffers, d_classes.py:1185-1224,
   * 1701-1807; quirk Q13).  NULL = synchronous schedule.                    */
  const uint8_t* zLag;      /* [R*K*K] 1: node k's update r consumes sender q's
                               fused frame of round r-1 instead of round r      */
  const double* zPhase;     /* [R*K*K] SRO phase-compensation offset phi (samples)
                               of sender q's channel at node k's update r:
                               yhat *= exp(-j 2 pi f phi / N) (compensate_sros,
                               d_classes.py:1936-2046); NULL = no compensation  */
  /* fewSamples broadcasts (broadcastType 'fewSamples' + efficientSpSBC: T(z)
   * compression of the last currL samples, d_classes.py:1090-1160,
   * d_base.py:1871-1991) instead of the wholeChunk WOLA compression.
   * NULL = wholeChunk.  Host-compiled by replaying the reference event order
   * (danse_amd/scheduler.py compile_rounds_fs); per (round r, node k):     */
  const int32_t* fsTab;     /* [R*K*DANSE_FS_FIELDS]: DANSE_FS_BCEND, _LEN, _POS,
                               _IRSRC, _ZEND (see enum danse_fs_field)          */
  int32_t zStreamLen;       /* samples per node stream with fsTab (else R*Ns)  */
  int32_t scmInitPerBin;    /* 1: scmInit holds one slice per bin, [F][D][D] per
                               family-node (covMatSameInitForAllFreqs = False,
                               init_from_wasn, d_classes.py:553-651); 0: [D][D] */
  /* CohDrift SRO estimation (estimateSROs 'CohDrift', closed loop, 'ls':
   * update_sro_estimates + build_phase_shifts_for_srocomp, d_classes.py:
   * 2364-2621; cohdrift_sro_estimation, d_sros.py:19-95).  The device keeps
   * the coherence ring, the averaged residual products and a per-(scene,
   * node, sender) phase accumulator that adds to zPhase (which then holds the
   * full-sample-drift flags only).  0 = off.                               */
  int32_t cohDrift;         /* 1: closed loop, 2: open loop (cohDrift.loop)     */
  int32_t cdSegLength;      /* segLength (ld)                                   */
  int32_t cdStart;          /* startAfterNups + estEvery (first estimate)       */
  int32_t cdEvery;          /* estEvery                                         */
  int32_t cdCompensate;     /* compensateSROs: accumulate the phase             */
  int32_t cdNIter;          /* the reference's nIter (estimation stops there)   */
  double cdAlpha;           /* alpha                                            */
  double cdAlphaEps;        /* alphaEps                                         */
  /* Centralised / single-sensor-broadcast observation vectors under
   * asynchronous clocks.  The reference sends every node's raw signals
   * through per-receiver buffers next to z (pre_fill_buffers_centralised /
   * fill_buffers_centr / process_incoming_signals_buffers_centr,
   * d_classes.py:1162-1183,1226-1250,1809-1891): receiver k's frame of sender
   * q is the last N samples of q's raw-signal stream, y_q[E - N, E).  The
   * device analyses that frame once per (round, sender) and the receivers
   * read it with the sender's zLag (0 without zLag).  NULL = synchronous: the
   * receivers use the senders' update-frame spectra.                        */
  const int32_t* cEnd;      /* [R*K] raw stream end E of sender q's round-r frame */
  const double* cPhase;     /* [R*K*MT] SRO phase offset (samples) of centralised
                               channel c at node k's update r (phaseShiftFactors-
                               Centr, compensate_sros d_classes.py:1996-2038 and
                               update_sro_estimates 2364-2621); NULL = none     */
  /* DXCP-PhaT SRO estimation in the loop (estimateSROs 'DXCPPhaT'; the
   * reference's own integration raises, d_classes.py:2469-2481, quirk Q12:
   * this is an extension).  One DXCP-PhaT estimator (sro_estimation.py:
   * 130-345, default parameters) per (scene, receiver k, sender q), fed every
   * 2048 / Ns rounds with the 2048 newest samples of k's reference sensor
   * (ending at upEnd[r][k]) and of q's fused-signal stream as k received it;
   * eps_kq = -(SRO ppm) 1e-6 replaces the Oracle estimate: with
   * cdCompensate the sender's phase loses eps Ns after every update.
   * wholeChunk broadcasts; exclusive with cohDrift.  0 = off.             */
  int32_t dxcp;
  /* Latency layout for small batches: 1 = the GEVD filter dimensions D <= 12
   * run on the 4 x 4 lane-grid solver (four bins per wavefront, full
   * [F][D][D] SCM storage) instead of one bin per lane: 16x the wavefronts,
   * for one or a few WASNs per GPU.  0 = one bin per lane (throughput).   */
  int32_t smallDGrid;
  /* fewSamples device steps (with fsTab): fsEv [nFsEv][K][DANSE_FS_FIELDS]
   * chunk rows (BCEND, LEN, POS, IRSRC; ZEND unused; LEN 0 and IRSRC -1 for
   * nodes without a chunk in that step), fsSteps [nFsSteps][DANSE_FS_STEP_
   * FIELDS] in execution order, round r's steps contiguous and in round
   * order.  NULL = one CHUNK (fsTab row r), BCAST, UPDATE per round.       */
  const int32_t* fsEv;
  int32_t nFsEv;
  const int32_t* fsSteps;
  int32_t nFsSteps;
  /* fewSamples with centralised / SSBC estimates under SRO clocks: 1 = the
   * centralised buffers receive each chunk's raw samples (the last currL of
   * the broadcast frame, pre_fill_buffers_centralised, d_classes.py:
   * 1162-1250) into per-channel streams with the z streams' positions, and
   * the receivers' raw frame of sender q is stream[cEnd - N, cEnd) -- the
   * frame ends floor(t fs) of consecutive chunks may overlap or skip a
   * sample, so the stream is not a slice of y.                           */
  int32_t rawStreams;
  /* desSigProcessingType 'conv' (get_desired_sig_chunk, d_base.py:2085-2100,
   * d_classes.py:2623-2709): 1 = every family's time-domain estimate is the
   * last Ns samples of the T(z) convolution of the first M_k channels of its
   * observation vector's update frame with the IRs dist_fct_approx(w[r + 1],
   * win_s, win_s, Ns) of the same filter columns, written to d[end - Ns,
   * end) (no overlap-add); dhat is NaN (the reference stores None).      */
  int32_t desSigConv;
  /* CohDrift open loop (cohDrift == 2; update_sro_estimates, d_classes.py:
   * 2376-2386,2439-2450; cohdrift_sro_estimation, d_sros.py:19-95): per
   * (round r, receiver k, sender q) broadcastLength * (sum of the buffer flags
   * of rounds r - segLength + 1 .. r) -- bufferFlagPos - bufferFlagPri, the
   * full-sample drifts inside the coherence segment, whose linear phase the
   * residual product loses; the coherence is taken on the UNcompensated
   * observation.  [R*K*K] doubles; NULL with the closed loop.              */
  const double* cdFlagWin;
} danse_cfg;

typedef struct danse_engine danse_engine;

/* Output identifiers for danse_engine_get(). Layouts (device order):
 *   DANSE_OUT_W      family f, node k: [S][R+1][F][D_fk] complex (2 slots if !keepHistory)
 *   DANSE_OUT_WEXT   node k: [S][R+1][F][M_k] complex
 *   DANSE_OUT_D      family f: [S][K][T] float (time-domain estimate)
 *   DANSE_OUT_DHAT   family f: [S][K][R][F] complex
 *   DANSE_OUT_Z      [S][K][R*Ns] float (zFullTD)
 *   DANSE_OUT_DIAG   [S*K*4] int32 diagnostics (bit0: non-PD pivot met in a solve) */
enum danse_output {
  DANSE_OUT_W = 0,
  DANSE_OUT_WEXT = 1,
  DANSE_OUT_D = 2,
  DANSE_OUT_DHAT = 3,
  DANSE_OUT_Z = 4,
  DANSE_OUT_DIAG = 5
};

/* Create / destroy.  `device` selects the HIP device. */
int danse_engine_create(const danse_cfg* cfg, int device, danse_engine** out);
void danse_engine_destroy(danse_engine* eng);
const char* danse_last_error(const danse_engine* eng);   /* eng may be NULL */
/* sha256 (hex) of the sources and flags this library was built from
 * (danse_amd/build.py source_hash); the Python side refuses a mismatch. */
const char* danse_mi355x_build_id(void);

/* Re-initialise all state (filters, SCMs, z streams, estimates) to the
 * configured initial values, asynchronously on `stream` (NULL: synchronous). */
int danse_engine_reset(danse_engine* eng, void* stream);

/* Borrow the input signals: device pointer to [S][sum_k M_k][T] float32,
 * channel order node-major (node 0 mics, node 1 mics, ...). */
int danse_engine_set_inputs(danse_engine* eng, const float* yDev);

/* Run rounds [r0, r1) on `stream` (hipStream_t; NULL = default stream).
 * graph != 0 captures the launch sequence in a hipGraph once and replays it. */
int danse_engine_run(danse_engine* eng, int32_t r0, int32_t r1, void* stream, int32_t graph);

/* The whole run in ONE persistent launch (the resident engine, SURVEY §8
 * row N1; the round loop of danse_toolbox/d_core.py:66-90 with every bin's
 * SCMs resident in registers and its GEVD factor in LDS): the WOLA analyses
 * of every round, round 0's broadcast, the persistent round loop (update
 * waves on 4 x 4 lane grids + one broadcast wave per (scene, node)), the
 * installed speculative gate checks (danse_engine_set_gate) and the estimate
 * synthesis, all on `stream`, no host synchronisation.  Needs: one engine
 * owning every node, wholeChunk broadcasts, no CohDrift / DXCP / centralised
 * raw frames, GEVD, every filter dimension <= 12 in full (grid) storage
 * (danse_cfg.smallDGrid), no pre-given filters, and the whole
 * grid resident at once (returns -1 with the reason otherwise).  A wait that
 * gives up sets the flag danse_engine_resident_error reads.             */
int danse_engine_run_resident(danse_engine* eng, void* stream);
int danse_engine_resident_error(danse_engine* eng, int32_t* err, void* stream);
/* Test hook: overwrite the give-up flag (every resident run clears it at
 * its start, so a stale flag never outlives the run that set it).       */
int danse_engine_resident_set_error(danse_engine* eng, int32_t value);
/* DXCP-PhaT in the loop (danse_cfg.dxcp): record every feed's gathered
 * estimator input frames and outputs, for checking the per-(receiver,
 * sender) estimators against the reference's DXCPPhaT
 * (dxcpphat/sro_estimation.py:117-345; d_sros.py:98-140 is the reference's
 * per-pair wrapper).  Pairs p = (s * nOwn + (k - k0)) * (K - 1) + qi, sender
 * q = qi < k ? qi : qi + 1; frames [nFeeds][P][2][2048] f32 (channel 0 the
 * receiver's reference sensor, channel 1 the sender's received z stream),
 * outputs [nFeeds][P][2] f64 (SRO ppm, STO samples).  _recorded reports the
 * sizes when the buffers are NULL.                                       */
/* Graph-safe device fill (every byte of [ptr, ptr + bytes) set to value &
 * 0xff, asynchronously on stream): a kernel, where a hipMemsetAsync captured
 * into a graph is not re-applied correctly by later launches of the graph
 * (DESIGN.md §6.2).  The engines fill their own state this way.          */
int danse_mi355x_fill(void* ptr, int32_t value, size_t bytes, void* stream);
int danse_engine_dxcp_record(danse_engine* eng, int32_t on);
int danse_engine_dxcp_recorded(danse_engine* eng, int32_t* nFeeds, int32_t* nPairs, float* frames,
                               size_t frameBytes, double* out, size_t outBytes);
/* Diagnostics: with DANSE_RESIDENT_TRACE set, the last resident run's
 * per-(round, wave) wall-clock marks ([R][waves][2] uint64, 100 MHz: after
 * the wait, at the publish); *bytes in: capacity of dst (may be NULL), out:
 * the size. */
int danse_engine_resident_trace(danse_engine* eng, void* dst, size_t* bytes);
/* Diagnostics of the warm-started rank-1 Lanczos path of the lane-grid GEVD
 * classes (update_w_gevd, d_classes.py:3343-3387, solved by solver2d.hpp
 * lanczos2d): per round of the last run, [R][2] int32 -- the bins whose warm
 * solve was accepted, and the bins the acceptance test sent back to the
 * Householder path.  n: capacity of dst in elements (>= 2 R). */
int danse_engine_lanczos_stats(danse_engine* eng, int32_t* dst, size_t n);

/* Condition numbers of Ryy (ConditionNumbers.get_new_cond_number,
 * d_classes.py:19-130,2126-2186; saveConditionNumber /
 * saveConditionNumberEvery): with every > 0, after the update of every round
 * r with (r + 1) % every == 0, np.linalg.cond of every (scene, family-node,
 * bin)'s Ryy (DANSE, local, centralised; NaN for SSBC).  danse_engine_cond
 * copies [S][family-nodes in engine order][R][F] float64 (NaN where not
 * saved) to host memory. */
int danse_engine_set_cond(danse_engine* eng, int32_t every);
int danse_engine_cond(danse_engine* eng, double* dst, size_t bytes);

/* Fine-grained per-round phases (multi-GPU: the caller all-gathers the fused
 * spectra between them).  bcast(r) also synthesises the estimates of r-1. */
int danse_engine_bcast(danse_engine* eng, int32_t r, void* stream);
int danse_engine_update(danse_engine* eng, int32_t r, void* stream);
int danse_engine_finish(danse_engine* eng, void* stream);
/* fewSamples engines: steps [s0, s1) of the compiled step list (danse_cfg.
 * fsSteps; round r's steps are contiguous), un-graphed and without the
 * speculative gate checks: the exact start gate of a round whose updates run
 * as several steps decides each node right before its own update step
 * (check_covariance_matrices, d_classes.py:1430-1540).  danse_engine_bcast /
 * _update of such an engine run round r's steps before / from its first
 * update step.                                                            */
int danse_engine_run_steps(danse_engine* eng, int32_t s0, int32_t s1, void* stream);
/* Node-sharded DXCP-PhaT (danse_cfg.dxcp on an engine owning [k0, k1) of
 * K nodes): the estimators of a receiver read every sender's received z
 * stream, i.e. the Ns new samples each node broadcasts per round
 * (fill_buffers, d_classes.py:1185-1224).  set_zchunk installs a [K][S][Ns]
 * float device buffer (node-major: this engine's nodes [k0, k1) are one
 * contiguous all-gather chunk) that every broadcast also writes; after the
 * all-gather of round r, unpack_zchunk copies the other nodes' chunks into
 * their streams.                                                          */
int danse_engine_set_zchunk(danse_engine* eng, void* ptr);
int danse_engine_unpack_zchunk(danse_engine* eng, int32_t r, void* stream);   /* synthesis of the last round */

/* Device pointer + byte size of the fused-signal spectra buffer [2][K][S][F]
 * complex: round r writes slot r & 1 (node-major within a slot, so that a
 * node range is one contiguous block); an update may read slot (r-1) & 1
 * (zLag). */
int danse_engine_zspec(danse_engine* eng, void** ptr, size_t* bytes);
/* The reference's start-of-updates gate (check_covariance_matrices,
 * d_classes.py:1430-1540) for n candidate (family, node, scene) triples at
 * round r, after danse_engine_bcast(r) and before danse_engine_update(r):
 * Hermitian (GEVD), positive definite and full rank over every bin, on the
 * SCMs after round r's recursion.  qY / qN: beta^m of the init slice's
 * anti-Hermitian residue in Ryy / Rnn (0 after a first-frame SET).
 * verdict[i] = 1 pass / 0 fail.  Synchronous (the host decides the flags).  */
int danse_engine_gate(danse_engine* eng, int32_t r, int32_t n, const int32_t* family, const int32_t* node,
                      const int32_t* scene, const double* qY, const double* qN, int32_t* verdict, void* stream);
/* Replace the round control table (same layout as danse_cfg.flags); the host
 * re-derives the solve flags when the gate delays a node's start.        */
int danse_engine_set_flags(danse_engine* eng, const uint8_t* flags, void* stream);
/* CohDrift outputs (SROsEstimates / SROsResiduals of the reference, rows of
 * the rounds run): est, res [S][K][R][K-1] double, host memory.           */
int danse_engine_sro_estimates(danse_engine* eng, double* est, double* res);
/* Speculative form of the gate for graph-captured runs: the n candidates
 * (round, family, node, scene, qY, qN) are checked inside danse_engine_run
 * (between bcast and update of their round) while the run proceeds on the
 * flags compiled for "every gate passes"; danse_engine_gate_verdicts
 * (synchronous) returns the verdicts in the order given, sorted stably by
 * round.  If one failed, the host re-runs with danse_engine_gate.          */
int danse_engine_set_gate(danse_engine* eng, int32_t n, const int32_t* round, const int32_t* family,
                          const int32_t* node, const int32_t* scene, const double* qY, const double* qN);
int danse_engine_gate_verdicts(danse_engine* eng, int32_t* verdict, void* stream);
/* The speculative gate of round r alone, for callers that sequence the
 * rounds themselves (the node-sharded runner: bcast(r), all-gather, then
 * this, then update(r)); r == 0 also re-arms the verdicts.  Asynchronous
 * and capturable (no host synchronisation).  Same check as inside
 * danse_engine_run (check_covariance_matrices, d_classes.py:1430-1540).   */
int danse_engine_gate_launch(danse_engine* eng, int32_t r, void* stream);
/* Use a caller-owned buffer (same size and layout) for the fused spectra,
 * e.g. a torch tensor that an RCCL all-gather fills in place. */
int danse_engine_set_zspec(danse_engine* eng, void* ptr);

/* Copy an output (enum danse_output) to `dst` (device or host pointer,
 * hipMemcpyDefault).  `family` selects the estimator family and `node` the
 * node for the per-node outputs (W, WEXT: all scenes, [S][...] contiguous);
 * both are ignored where irrelevant.  Synchronises `stream`. */
int danse_engine_get(danse_engine* eng, int32_t which, int32_t family, int32_t node, void* dst, size_t bytes,
                     void* stream);
/* Inverse of danse_engine_get for DANSE_OUT_W / DANSE_OUT_WEXT: load a full
 * filter history (the SNR replay with pre-given filters). */
int danse_engine_put(danse_engine* eng, int32_t which, int32_t family, int32_t node, const void* src, size_t bytes,
                     void* stream);
/* Byte size of an output. */
int danse_engine_output_bytes(danse_engine* eng, int32_t which, int32_t family, int32_t node, size_t* bytes);

/* ---- fine-grained operators, for tests and other callers ---- */

/* WOLA analysis (build_ytilde, d_classes.py:1927-1934):
 * out[c][F] = FFT(x[c][end-N:end] * win)[:F] / sqrt(Ns), zero-padded before 0.
 * x: [C][T] float (device), ends: [C] int32 (device), out: [C][F] complex. */
int danse_wola_analysis(const float* x, int32_t C, int32_t T, const int32_t* ends,
                        const float* win, int32_t N, int32_t Ns, float* out, void* stream);

/* Whole-signal STFT (the reference's yinSTFT / yCentrBatch, d_classes.py:
 * 915-930: scipy.signal.stft(boundary=None, padded=True) times sum(win), i.e.
 * raw windowed DFTs of frames t Ns .. t Ns + N, zero past the end):
 * y: [S][C][T] float (device), win: [N] float (device),
 * out: [S][F][nseg][C] complex float (device), F = N/2 + 1.  N = 1024. */
int danse_stft(const float* y, int32_t S, int32_t C, int32_t T, int32_t N, int32_t Ns, int32_t nseg,
               const float* win, float* out, void* stream);

/* Batched filter update on full SCM pairs (update_w / update_w_gevd,
 * d_classes.py:3320-3387): Ryy, Rnn: [B][D][D] complex double (device), w:
 * [B][D] complex float.  The SCM the update factors (Rnn for GEVD, Ryy for
 * MWF) is used in double, the other one in float (DESIGN.md "Precision").
 * gevd != 0 -> rank-`rank` GEVD, else MWF. diag: [B] int32 or NULL. */
int danse_filter_update(const double* Ryy, const double* Rnn, int32_t B, int32_t D, int32_t gevd,
                        int32_t rank, int32_t ref, float* w, int32_t* diag, void* stream);

/* Batch-mode SCM contraction (update_covmats_batch, d_classes.py:3272-3304):
 * Y: [B][Tf][D] complex, vad: [Tf] uint8 (device) -> Ryy, Rnn: [B][D][D]
 * complex (means over VAD / non-VAD frames; MFMA f32 HERK). */
int danse_batch_covmats(const float* Y, int32_t B, int32_t Tf, int32_t D, const uint8_t* vad,
                        float* Ryy, float* Rnn, void* stream);

/* ---- batch-mode engine (danse_batch, d_core.py:251-352; d_batch.py) ----
 * Replaces the reference's danse_batch(wasnObj, p): STFT of the whole
 * signal, then maxBatchUpdates iterations of z = wExt^H y, Y.Y^H SCMs over
 * VAD / non-VAD frames, MWF / GEVD filter update (seq: one node per
 * iteration, asy/sim: all), external filters, dhat = w^H ytilde, ISTFT and
 * the MMSE cost.  Fully connected, DANSE estimates only. */
typedef struct danse_batch_cfg {
  int32_t S;               /* scenes (same shape)                                 */
  int32_t K;               /* nodes                                               */
  const int32_t* M;        /* [K] sensors per node                                */
  int32_t N, Ns, T;        /* DFT size (1024), hop, samples per channel           */
  int32_t iters;           /* maxBatchUpdates                                     */
  int32_t nseg;            /* STFT frames of the end-padded signal (scipy padded=True) */
  int32_t gevd, rank, ref;
  float alphaExt;          /* alphaExternalFilters                                */
  const int32_t* extMode;  /* [K] enum danse_ext_mode                             */
  const float* betaExt;    /* [S*K] external-filter forgetting factors            */
  const float* win;        /* [N] STFT window (winWOLAanalysis)                   */
  const uint8_t* vad;      /* [S][K][nseg] frame VAD (WASN.get_vad_per_frame)     */
  const uint8_t* doSolve;  /* [iters][K] 1: node updates its filters this iteration */
  const float* w0;         /* initial filters, node blocks [F][D_k] complex        */
  const float* wExt0;      /* initial external filters (and targets), [F][M_k]     */
  int32_t costTrim;        /* samples trimmed at both ends in the MMSE cost (1000) */
  int32_t k0, k1;          /* owned nodes [k0, k1) (node-sharded batch DANSE across
                              GPUs: z for every node, SCMs / solves / estimates /
                              cost for the owned ones); k1 <= k0: all nodes     */
  const float* tgt0;       /* initial external-filter targets (wTildeExtTarget,
                              d_classes.py:702-708), layout of wExt0; NULL: wExt0 */
  int32_t obs;             /* observation vector: 0 DANSE (local mics + the other
                              nodes' z), 1 local (the node's own mics), 2
                              centralised (every sensor of the WASN, reference
                              index sum(M[:k]) + ref): the batch centralised /
                              local estimates (get_centralized_and_local_estimates,
                              d_batch.py:20-88) and the best-performance
                              reference (get_best_perf, d_core.py:602-627;
                              get_centralized_estimates, d_batch.py:90-125).
                              With obs != 0 there are no z and no external
                              filters; doSolve = 0 keeps the pre-given w0.    */
} danse_batch_cfg;

typedef struct danse_batch danse_batch;

/* Outputs of danse_batch_get:
 *   W     node k: [S][iters+1][F][D_k] complex     WEXT node k: [S][iters+1][F][M_k]
 *   D     [S][K][T] float (last iteration)          DHAT [S][K][nseg-1][F] complex
 *   COST  [iters][S][K] double (NaN-free only when clean signals were given) */
enum danse_batch_output {
  DANSE_BATCH_OUT_W = 0,
  DANSE_BATCH_OUT_WEXT = 1,
  DANSE_BATCH_OUT_D = 2,
  DANSE_BATCH_OUT_DHAT = 3,
  DANSE_BATCH_OUT_COST = 4
};

int danse_batch_create(const danse_batch_cfg* cfg, int device, danse_batch** out);
void danse_batch_destroy(danse_batch* eng);
const char* danse_batch_last_error(const danse_batch* eng);
/* y: [S][sum_k M_k][T] float (device); clean: [S][K][T] float (device, the
 * clean speech at each node's reference sensor) or NULL (no MMSE cost). */
int danse_batch_set_inputs(danse_batch* eng, const float* y, const float* clean);
int danse_batch_run(danse_batch* eng, void* stream);
/* Iterations [it0, it1) (it0 == 0 also sets the initial state and the STFT);
 * between two calls a node-sharded run exchanges the external filters of
 * slot it1 (written by iteration it1 - 1):
 *   danse_batch_pack_wext(own nodes -> dst [k1-k0][S][F*Mmax] complex),
 *   all-gather over ranks into [K][S][F*Mmax],
 *   danse_batch_unpack_wext(the other nodes' slots <- src).
 * (update_external_filters_batch + batch z, d_core.py:286-326)          */
int danse_batch_run_iters(danse_batch* eng, int32_t it0, int32_t it1, void* stream);
int danse_batch_pack_wext(danse_batch* eng, int32_t slot, void* dst, void* stream);
int danse_batch_unpack_wext(danse_batch* eng, int32_t slot, const void* src, void* stream);
int danse_batch_output_bytes(danse_batch* eng, int32_t which, int32_t node, size_t* bytes);
int danse_batch_get(danse_batch* eng, int32_t which, int32_t node, void* dst, size_t bytes, void* stream);
/* Per-phase device timing of danse_batch_run_iters (HIP events recorded on
 * the run's stream at every phase boundary of every iteration, off by
 * default).  danse_batch_timing sums iterations [it0, it1) of the last run
 * into ms[7]: z, Y.Y^H (HERK), solves, external filters, dhat, ISTFT + OLA,
 * MMSE cost.  Synchronous (waits for iteration it1 - 1).                     */
int danse_batch_set_timing(danse_batch* eng, int32_t on);
int danse_batch_timing(danse_batch* eng, int32_t it0, int32_t it1, float* ms);

/* ---- DXCP-PhaT sampling-rate-offset estimator (dxcpphat/sro_estimation.py:
 * 130-345, class DXCPPhaT with its default parameters: fs 16 kHz, 2048-sample
 * frames, 8192-point FFT, 5 s accumulation), batched over P node pairs.
 * danse_dxcp_process() is one process_data() call of every pair:
 *   x:   [P][2][2048] float (device): the two channels' next frame
 *   out: [P][2] double (device): SROppm_est_out, STOsmp_est_out after it. */
typedef struct danse_dxcp danse_dxcp;
int danse_dxcp_create(int32_t P, int device, danse_dxcp** out);
void danse_dxcp_destroy(danse_dxcp* eng);
const char* danse_dxcp_last_error(const danse_dxcp* eng);
int danse_dxcp_process(danse_dxcp* eng, const float* x, double* out, void* stream);
/* Every pair back to its initial state (asynchronous on `stream`).         */
int danse_dxcp_reset(danse_dxcp* eng, void* stream);
/* process_data(x_12_ell, tdoa): as danse_dxcp_process, with the STO
 * estimate corrected by tdoa[p] * 16000 samples when its maximum is interior
 * (sro_estimation.py:338-339).  tdoa: [P] double (device) or NULL.        */
int danse_dxcp_process_tdoa(danse_dxcp* eng, const float* x, const double* tdoa, double* out, void* stream);
/* Closed-loop DXCP-PhaT (class CL_DXCPPhaT, sro_estimation.py:12-72) for P
 * pairs: per frame the OnlineResampler (online_resampler.py:4-77) of z_i by
 * -SRO_est_curr, the 3-frame DelayBuffer (delay_buffer.py:8-26) of z_j,
 * DXCP-PhaT on the synchronised pair and the IMC controller (PIT1, Tf = 8;
 * frozen for ell <= startDelay).  Engines from danse_cl_dxcp_create are
 * danse_dxcp handles (danse_dxcp_destroy frees them).
 *   x:   [P][2][2048] float (device): z_j (reference) then z_i
 *   acs: [P] int32 (device) or NULL (all 1): 0 forces the residual to 0
 *   out: [P][3] double (device): dSRO_est_curr_raw, SRO_est_curr,
 *        Resampler.shift after the call (the process() return values)
 *   zi:  [P][2048] float (device) or NULL: the synchronised z_i block
 *        (from two calls earlier)                                          */
int danse_cl_dxcp_create(int32_t P, int32_t startDelay, int device, danse_dxcp** out);
int danse_cl_dxcp_process(danse_dxcp* eng, const float* x, const int32_t* acs, double* out, float* zi, void* stream);

/* ---- Synthetic scenes on the device (csrc/scene.hip):
 * the random-IR / random-signal path of siggen (build_wasn, siggen/utils.py:
 * 1155-1411, trueRoom false, signalType random) for S scenes at once --
 * paused uniform desired source and uniform noise source per scene, uniform
 * random IRs per sensor (causal convolution), noise gain for `snr` at mic 0
 * of node 0, per-node SRO resampling to fs (1 + sroPpm 1e-6) by a Kaiser-
 * windowed sinc (resample_for_sro, utils.py:1579-1622, uses resampy, absent
 * offline: parity unpinned), sensor self-noise at selfnoiseSNR
 * (apply_self_noise, utils.py:1414-1431), energy VAD of each node's mic-0 wet
 * speech.  Random numbers: counter-based (seed + scene, stream, index).
 * Outputs (device): data, cleanspeech, cleannoise [S][sum M][T] float,
 * vad [S][K][T] uint8.  Synchronises `stream`.                           */
typedef struct danse_scene_cfg {
  int32_t S, K;
  const int32_t* M;         /* [K] sensors per node                            */
  int32_t T;                /* samples per channel                             */
  int32_t nIR;              /* IR taps (randIRsParams.duration * fs)           */
  int64_t seed;             /* scene s uses seed + s                           */
  double fs, snr, selfnoiseSNR, pauseDuration, pauseSpacing;
  double vadEnergyDecrease_dB, vadWinLength;
  const double* sroPpm;     /* [K] or NULL                                     */
} danse_scene_cfg;
const char* danse_scene_last_error(void);
int danse_scene_generate(const danse_scene_cfg* cfg, float* data, float* cleanspeech, float* cleannoise, uint8_t* vad,
                         void* stream);
/* The generator's convolution and VAD kernels on injected rows (device
 * pointers): out[r] = (x[r] * h[r])[:T] (the wet signals of build_wasn,
 * sig.fftconvolve(xdry, rir)[:T], siggen/utils.py:867-872) and, if vad is
 * not NULL, vad[r] = oracleVAD(out[r], vadWinLength, max(out[r]^2) /
 * 10^(dB/10), fs) (siggen/utils.py:896-939,1079-1151).  x, out [rows][T]
 * float, h [rows][nIR] float, vad [rows][T] uint8.  Synchronises stream. */
int danse_scene_convolve_vad(const float* x, const float* h, int32_t rows, int32_t T, int32_t nIR, float* out,
                             double vadWinLength, double fs, double vadEnergyDecrease_dB, uint8_t* vad,
                             void* stream);

/* ---- T(z) few-samples compression (broadcastType 'fewSamples').
 * danse_tz_create: analysis window h, synthesis window f (N floats, host), the
 *   WOLA shift R (= Ns); N = 1024.
 * danse_tz_ir replaces dist_fct_approx(wHat, h, f, R) (danse_toolbox/
 *   d_base.py:1941-1991) for B filters at once:
 *     wHat: [B][N/2+1][M] complex float (device; the reference's wqqHat layout)
 *     wIR:  [B][2N-1][M] float (device; the reference's wIR layout).
 * danse_tz_compress replaces the convolution of danse_compression_few_samples
 *   (d_base.py:1871-1938, extract_few_samples_from_convolution 1538-1566):
 *     yq:   [B][N][M] float (device; each node's local frame ykFrame)
 *     wIR:  [B][2N-1][M] float (device)
 *     z:    [B][L] float (device): the last L samples of the T(z)-filtered
 *           frame summed over the node's sensors (zq), 1 <= L <= N. */
typedef struct danse_tz danse_tz;
int danse_tz_create(int32_t N, const float* h, const float* f, int32_t R, int device, danse_tz** out);
void danse_tz_destroy(danse_tz* eng);
const char* danse_tz_last_error(const danse_tz* eng);
int danse_tz_ir(danse_tz* eng, const float* wHat, int32_t B, int32_t M, float* wIR, void* stream);
int danse_tz_compress(danse_tz* eng, const float* yq, const float* wIR, int32_t B, int32_t M, int32_t L, float* z,
                      void* stream);

/* ---- Enhancement metrics, float64 (csrc/metrics.hip).
 * danse_snr replaces get_snr(s, n, vad) (danse_toolbox/d_eval.py:573-624):
 *     s, n: [C][T] double (device; the reference's [T x C] transposed)
 *     vad:  [C][T] uint8 (device) or NULL (bypassVADuse: whole signal)
 *     out:  [C] double (device): 10 log10(mean s^2 / mean n^2) over vad.
 * danse_fwsnrseg replaces get_fwsnrseg(clean, enhanced, fs, frameLen,
 *   overlap, gamma) (d_eval.py:660-778) for nSig signal pairs at once:
 *     clean, enhanced: [nSig][T] double (device)
 *     perFrame: [nSig][nFrames] double (device): the clipped per-frame values
 *     mean:     [nSig] double (device) or NULL: np.mean over frames (the
 *               fwSNRseg.before / .after of get_metrics, d_eval.py:236-244).
 * danse_fwsnrseg_frames gives nFrames = int(T / skip - W / skip).         */
const char* danse_metrics_last_error(void);
int danse_snr(const double* s, const double* n, const uint8_t* vad, int64_t T, int32_t C, double* out, void* stream);
int danse_fwsnrseg_frames(int64_t T, double fs, double frameLen, double overlap, int32_t* nFrames);
int danse_fwsnrseg(const double* clean, const double* enhanced, int64_t T, int32_t nSig, double fs, double frameLen,
                   double overlap, double gamma, double* perFrame, double* mean, void* stream);

/* (e)STOI, float64 (csrc/stoi.hip) for nSig (clean, processed) pairs,
 * replacing stoi / stoi_any_fs (danse_toolbox/mypystoi/stoi.py:18-239, the
 * 'stoi' entry of get_metrics, d_eval.py:254-331, uses extended = True):
 *     x, y: [nSig][T] double (device), fs: integer sampling rate
 *     out:  [nSig] double (device)
 * At fs != 10000 both signals are resampled to 10 kHz with the Octave
 * resampler of mypystoi utils.resample_oct (utils.py:8-47), as stoi() does;
 * stoi_any_fs resamples with resampy instead (absent offline: unpinned).
 * Fewer than 30 STFT frames after silent-frame removal give 1e-5, as the
 * reference.  Synchronises `stream` (scratch buffers).                 */
const char* danse_stoi_last_error(void);
int danse_stoi(const double* x, const double* y, int64_t T, int32_t nSig, double fs, int32_t extended, double* out,
               void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DANSE_MI355X_H */
