/*
 * danse_mi355x_defs.h -- the constants of the C-ABI (include/danse_mi355x.h)
 * that the device kernels also read: estimator families, round control
 * bytes, external-filter modes, fewSamples schedule fields.  Kept apart so
 * that the kernel translation units do not depend on the entry points.
 */
#ifndef DANSE_MI355X_DEFS_H
#define DANSE_MI355X_DEFS_H

#define DANSE_MAX_FAMILIES 4   /* DANSE, local, centralised, single-sensor broadcast */

enum danse_family {
  DANSE_FAM_DANSE = 0,   /* wTilde / d / dhat                 d_classes.py:2290-2320 */
  DANSE_FAM_LOCAL = 1,   /* wLocal / dLocal                   d_classes.py:2339-2350 */
  DANSE_FAM_CENTR = 2,   /* wCentr / dCentr                   d_classes.py:2321-2338 */
  DANSE_FAM_SSBC = 3     /* wSSBC / dSSBC                     d_classes.py:2351-2362 */
};

/* Per-round, per-(scene, family, node) control byte (host-computed schedule).
 * bits 0-1: Ryy op   bits 2-3: Rnn op   (0 keep, 1 set to yy^H, 2 exp. average)
 *           (spatial_covariance_matrix_update + conditional_scm_updating,
 *            d_classes.py:2048-2267)
 * bit 4   : solve (filter update: not bypassed and gate passed,
 *           d_classes.py:1298-1313 / 2290-2362); else w[i+1] = w[i]
 * bit 5   : refresh the asy external-filter target (timeBtwExternalFiltUpdates,
 *           d_classes.py:1680-1694)                                         */
#define DANSE_OP_KEEP 0
#define DANSE_OP_SET 1
#define DANSE_OP_AVG 2
#define DANSE_FLAG_SOLVE 0x10
#define DANSE_FLAG_EXT_TARGET 0x20
#define DANSE_FLAG_PREGIVEN 0x40   /* w[i+1], wExt[i+1] pre-loaded (danse_engine_put):
                                      update_using_pregiven_filters, d_classes.py:1338-1352 */
#define DANSE_FLAG_INITSLOT 0x80   /* the family-node has not started updating: its filter
                                      for this round is the (pre-loaded) init slot w[i+1]
                                      (perform_update leaves wTilde[:, i+1] untouched,
                                      d_classes.py:2290-2362; differs from w[i] only for
                                      filterInitType 'random') */

/* External-filter update mode per node (update_external_filters,
 * d_classes.py:1627-1694). */
enum danse_ext_mode {
  DANSE_EXT_COPY = 0,    /* seq or noExternalFilterRelaxation: wExt[i+1] = w[i+1][:M]     */
  DANSE_EXT_RELAX = 1,   /* asy/sim: wExt[i+1] = b wExt[i] + (1-b) target; target update */
  DANSE_EXT_KEEP = 2,    /* noFusionAtSingleSensorNodes and M_k == 1                      */
  DANSE_EXT_REFONLY = 3  /* onlyBroadcastRefSensorSigs                                    */
};

/* Fields of one fsTab entry (round r, node k). */
enum danse_fs_field {
  DANSE_FS_BCEND = 0,   /* broadcast frame end floor(t fs) of node k's broadcast in round r */
  DANSE_FS_LEN = 1,     /* currL: samples appended to node k's stream (0: none)             */
  DANSE_FS_POS = 2,     /* stream position of that chunk                                    */
  DANSE_FS_IRSRC = 3,   /* >= 0: refresh the T(z) IR from wExt iteration IRSRC first
                           (upTDfilterEvery timer); -1: keep the current IR                 */
  DANSE_FS_ZEND = 4,    /* node k's stream length the receivers' round-r z frame ends at
                           (their frame = stream[ZEND - N, ZEND), zero before 0)            */
  DANSE_FS_FIELDS = 5
};

/* One fewSamples device step (danse_cfg.fsSteps, DANSE_FS_STEP_FIELDS int32):
 * type, round r, node mask (bit k: node k), chunk row (fsEv row of a CHUNK
 * step, else -1).  A round is a list of steps that keeps every dependency of
 * the reference's event order (danse_amd/scheduler.py compile_rounds_fs).   */
enum danse_fs_step {
  DANSE_FS_STEP_CHUNK = 0,   /* T(z) IR refresh + currL chunk append of the row's nodes */
  DANSE_FS_STEP_BCAST = 1,   /* round r's analyses, estimate synthesis of round r-1 and
                                the z frames of the masked senders                     */
  DANSE_FS_STEP_ZAN = 2,     /* z frames of the masked senders only                   */
  DANSE_FS_STEP_UPDATE = 3,  /* update r of the masked nodes                          */
  DANSE_FS_STEP_FIELDS = 4
};

#endif /* DANSE_MI355X_DEFS_H */
