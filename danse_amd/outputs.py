"""The ``dv`` output fields the reference's post-processing reads, and its
output container.

* ``host_fields``: the bookkeeping fields of ``DANSEvariables`` that follow
  from the schedule alone (SRO estimates / residuals with Oracle SROs, buffer
  flag iterations, the first-update instant, the never-filled online MSE
  cost arrays), restating ``d_classes.py:810-846,959-964,1271-1274,
  1955-1970,2364-2489,2562-2600``;
* ``DANSEoutputs``: ``d_post.DANSEoutputs.from_variables`` /
  ``from_snr_signals`` (``d_post.py:38-150``) field mapping.

Every array here is small host bookkeeping; the signal-sized fields (``d``,
``dhat``, filters, ``zFullTD``, ``yinSTFT``) come from the device
(``engine.DanseEngine.outputs``).
"""
from __future__ import annotations

import warnings

import numpy as np

# every attribute DANSEoutputs.from_variables (d_post.py:41-133) and
# d_core.format_output (d_core.py:105-127) read from an online ``dv``
ONLINE_DV_FIELDS = (
    'yin', 'd', 'dhat', 'zFullTD', 'SROsppm', 'SROsEstimates', 'SROsResiduals', 'flagIterations',
    'firstDANSEupdateRefSensor', 'wTilde', 'wTildeExt', 'yinSTFT', 'yCentrBatch', 'neighbors', 'fs',
    'cleanSpeechSignalsAtNodes', 'mseCostOnline', 'expAvgBeta', 'oVADframes',
    'computeCentralised', 'computeLocal', 'computeSingleSensorBroadcast',
)
# ... when the corresponding family is computed
FAMILY_DV_FIELDS = {
    'computeCentralised': ('dCentr', 'dHatCentr', 'wCentr', 'mseCostOnline_c'),
    'computeLocal': ('dLocal', 'dHatLocal', 'wLocal', 'mseCostOnline_l'),
    'computeSingleSensorBroadcast': ('dSSBC', 'dHatSSBC'),
}


def stft_frames(T: int, N: int, Ns: int) -> int:
    """Frames of ``scipy.signal.stft(..., boundary=None, padded=True)``: the
    signal is zero-padded at the end to a whole number of hops."""
    nadd = (-(T - N) % Ns) % N
    return (T + nadd - N) // Ns + 1


def host_fields(p, sros, neighbors, rt, nIter, nFramesSTFT, firstSolveRound):
    """Schedule-derived ``dv`` fields of one scene.

    sros           node SROs [ppm] (``dv.SROsppm``)
    neighbors      per node, its neighbour list
    rt             scheduler.RoundTables (update instants ``t[r, k]`` and
                   buffer flags ``flags[r, k, q]``)
    nIter          the reference's iteration count (array rows)
    nFramesSTFT    frames of ``yinSTFT`` (rows of the MSE cost arrays)
    firstSolveRound  round of the first DANSE filter update of node
                   ``p.referenceSensor`` (-1: none)
    """
    K, R = len(neighbors), rt.nRounds
    sros = np.asarray(sros, dtype=np.float64)
    out = {}
    # update_sro_estimates / build_phase_shifts_for_srocomp (d_classes.py:
    # 2364-2489, 2562-2600): with Oracle estimation every update writes the
    # residual row; with compensation also the estimate row
    est, res = [], []
    for k in range(K):
        nb = list(neighbors[k])
        e = np.zeros((nIter, len(nb)))
        s = np.zeros((nIter, len(nb)))
        if p.estimateSROs == 'Oracle':
            s[:R, :] = (sros[nb] - sros[k]) * 1e-6
            if p.compensateSROs:
                e[:R, :] = s[:R, :]
        est.append(e)
        res.append(s)
    if p.estimateSROs not in ('Oracle', 'CohDrift'):
        # DXCP-PhaT inside DANSE raises in the reference itself (quirk Q12)
        warnings.warn(f'estimateSROs={p.estimateSROs!r}: SROsEstimates / SROsResiduals are not computed')
        est, res = None, None
    # (CohDrift: the engine overwrites both with the device estimates)
    out['SROsEstimates'], out['SROsResiduals'] = est, res
    # compensate_sros (d_classes.py:1955-1970): one entry per neighbour whose
    # buffer flag is nonzero at that update
    flags = rt.flags
    fi = [[] for _ in range(K)]
    if flags is not None:
        for k in range(K):
            nb = list(neighbors[k])
            for r in range(R):
                for q in nb:
                    if flags[r, k, q] != 0:
                        fi[k].append(r)
    out['flagIterations'] = fi
    # update_and_estimate (d_classes.py:1271-1274) compares the NODE index
    # with referenceSensor: the update instant of that node up to (and
    # including) its first internal filter update
    kr = p.referenceSensor
    first = None
    if kr < K and R > 0:
        r = firstSolveRound if firstSolveRound >= 0 else R - 1
        first = float(rt.t[r, kr])
    out['firstDANSEupdateRefSensor'] = first
    # d_classes.py:959-964: allocated, never filled (compute_batch_mse_cost is
    # not called anywhere in the reference)
    mse = np.full((nFramesSTFT, K), fill_value=None)
    out['mseCostOnline'] = mse
    out['mseCostOnline_c'] = mse.copy()
    out['mseCostOnline_l'] = mse.copy()
    return out


class DANSEoutputs:
    """``d_post.DANSEoutputs`` (``d_post.py:22-150``): the parameters plus
    the output fields selected from ``dv``."""

    def __init__(self):
        self.initialised = False

    def import_params(self, p):
        self.__dict__.update(p.__dict__)
        return self

    def from_variables(self, dv):
        for nm in ('TDdesiredSignals_est_c', 'STFTDdesiredSignals_est_c', 'TDdesiredSignals_est_l',
                   'STFTDdesiredSignals_est_l', 'TDdesiredSignals_est_ssbc', 'STFTDdesiredSignals_est_ssbc',
                   'TDfiltSpeech_c', 'STFTfiltSpeech_c', 'TDfiltNoise_c', 'STFTfiltNoise_c', 'TDfiltSpeech_l',
                   'STFTfiltSpeech_l', 'TDfiltNoise_l', 'STFTfiltNoise_l', 'TDfiltSpeech_ssbc',
                   'STFTfiltSpeech_ssbc', 'TDfiltNoise_ssbc', 'STFTfiltNoise_ssbc'):
            setattr(self, nm, None)
        self.micSignals = dv.yin
        if self.simType == 'batch':
            self.mmseCost = dv.mmseCost
            self.mmseCostInit = dv.mmseCostInit
            if self.computeLocal:
                self.mmseCostLocal = dv.mmseCostLocal
            if self.computeCentralised:
                self.mmseCostCentr = dv.mmseCostCentr
        self.TDdesiredSignals_est = dv.d
        self.STFTDdesiredSignals_est = dv.dhat
        if self.computeCentralised:
            self.TDdesiredSignals_est_c = dv.dCentr
            self.STFTDdesiredSignals_est_c = dv.dHatCentr
        if self.computeLocal:
            self.TDdesiredSignals_est_l = dv.dLocal
            self.STFTDdesiredSignals_est_l = dv.dHatLocal
        if self.computeSingleSensorBroadcast:
            self.TDdesiredSignals_est_ssbc = dv.dSSBC
            self.STFTDdesiredSignals_est_ssbc = dv.dHatSSBC
        self.TDfusedSignals = dv.zFullTD
        if hasattr(dv, 'etaMkFullTD'):
            self.TDfusedSignalsTI = dv.etaMkFullTD
        self.SROgroundTruth = dv.SROsppm
        self.SROsEstimates = dv.SROsEstimates
        self.SROsResiduals = dv.SROsResiduals
        self.flagIterations = dv.flagIterations
        self.firstUpRefSensor = dv.firstDANSEupdateRefSensor
        self.filters = dv.wTilde
        if self.simType == 'online':
            self.filtersEXT = dv.wTildeExt
            self.yinSTFT = dv.yinSTFT
            self.yCentrBatch = dv.yCentrBatch
            self.neighbors = dv.neighbors
            self.fs = dv.fs
            self.cleanTargets = dv.cleanSpeechSignalsAtNodes
            self.mseCostOnline = dv.mseCostOnline
            if self.computeCentralised:
                self.mseCostOnline_c = dv.mseCostOnline_c
            if self.computeLocal:
                self.mseCostOnline_l = dv.mseCostOnline_l
        self.filtersCentr = dv.wCentr if self.computeCentralised else None
        self.filtersLocal = dv.wLocal if self.computeLocal else None
        if getattr(self, 'saveConditionNumber', False):
            self.condNumbers = dv.condNumbers
        self.beta = dv.expAvgBeta
        self.vadFrames = dv.oVADframes
        self.initialised = True
        return self

    # ---- disk formats (d_post.py:184-212,
    # dataclass_methods.py:13-117): <folder>/DANSEoutputs.pkl.gz (gzip'ed
    # pickle of the object), <folder>/DANSEoutputs_text.txt (one line per
    # field, nested objects indented) and <folder>/metrics.pkl
    def check_init(self):
        """``check_init`` (d_post.py:184-187): returns (does not raise) the
        error of an empty object, as the reference does."""
        if not self.initialised:
            return ValueError('The DANSEoutputs object is empty.')

    def save(self, foldername, light=False, exportType='pkl'):
        """``save`` (d_post.py:189-199).  With ``light`` the reference strips
        the '*signal*' fields from a copy and then saves the full object
        anyway; kept as such."""
        _save(self, foldername, exportType=exportType)

    def save_metrics(self, foldername):
        """``save_metrics`` (d_post.py:201-205): ``self.metrics`` pickled to
        <folder>/metrics.pkl."""
        self.check_init()
        import pickle
        with open(f'{foldername}/metrics.pkl', 'wb') as f:
            pickle.dump(self.metrics, f)

    def load(self, foldername, dataType='pkl'):
        """``load`` (d_post.py:207-209, dataclass_methods.py:45-95): the
        object this class saved to <folder>/DANSEoutputs.pkl.gz."""
        return _load(self, foldername, dataType=dataType)

    def from_snr_signals(self, snrSigs: dict):
        self.TDfiltSpeech = snrSigs['s']
        self.TDfiltNoise = snrSigs['n']
        self.TDfiltSpeech_c = snrSigs['s_c']
        self.TDfiltNoise_c = snrSigs['n_c']
        self.TDfiltSpeech_l = snrSigs['s_l']
        self.TDfiltNoise_l = snrSigs['n_l']
        self.TDfiltSpeech_ssbc = snrSigs['s_ssbc']
        self.TDfiltNoise_ssbc = snrSigs['n_ssbc']
        return self

    def include_best_perf_data(self, outBP, sigsSnr: dict):
        """``DANSEoutputs.include_best_perf_data`` (``d_post.py:152-182``):
        the best-performance reference (``core.get_best_perf``)."""
        self.bestPerfData = {
            'dCentr': outBP.dCentr,
            'dHatCentr': outBP.dHatCentr,
            'dCentr_s': sigsSnr['s_bp'],
            'dCentr_n': sigsSnr['n_bp'],
            'mseCostCentr': outBP.mmseCostCentr,
            'wCentr': outBP.wCentr,
            'fs': outBP.baseFs,
            'cleanSpeech': np.array([outBP.cleanSpeechSignalsAtNodes[k][:, outBP.referenceSensor]
                                     for k in range(outBP.nNodes)]).T,
            'cleanNoise': np.array([outBP.cleanNoiseSignalsAtNodes[k][:, outBP.referenceSensor]
                                    for k in range(outBP.nNodes)]).T,
        }
        return self


def _save(obj, foldername, exportType='pkl'):
    """``dataclass_methods.save`` (dataclass_methods.py:13-42): the gzip'ed
    pickle (or JSON, which raises in the reference: NOT YET CORRECTLY
    IMPLEMENTED) plus the text view."""
    import gzip
    import pickle
    from pathlib import Path
    Path(foldername).mkdir(parents=True, exist_ok=True)
    full = f'{foldername}/{type(obj).__name__}'
    if exportType == 'pkl':
        with gzip.open(full + '.pkl.gz', 'wb') as f:
            pickle.dump(obj, f)
    elif exportType == 'json':
        raise ValueError('NOT YET CORRECTLY IMPLEMENTED')
    _save_as_txt(obj, foldername)


def _load(obj, foldername, dataType='pkl'):
    """``dataclass_methods.load`` (dataclass_methods.py:45-95), for the
    files ``_save`` wrote (this package's own pickles only)."""
    import gzip
    import pickle
    from pathlib import Path
    if not Path(foldername).is_dir():
        raise ValueError(f'The folder "{foldername}" cannot be found.')
    base, alt = ('.pkl.gz', '.json') if dataType == 'pkl' else ('.json', '.pkl.gz')
    path = f'{foldername}/{type(obj).__name__}{base}'
    if not Path(path).is_file():
        other = f'{foldername}/{type(obj).__name__}{alt}'
        if not Path(other).is_file():
            raise ValueError(f'Import issue, file\n"{path}"\nnot found (with either possible extensions).')
        path, base = other, alt
    if base == '.json':
        raise ValueError('NOT YET CORRECTLY IMPLEMENTED')
    with gzip.open(path, 'rb') as f:
        return pickle.load(f)


def _save_as_txt(obj, foldername):
    """``save_as_txt`` (dataclass_methods.py:97-117): one ' - name = value'
    line per field, nested parameter objects indented with ' |'."""
    def lines(o, f, n=0):
        tab = ' |' * n
        f.write(f'{tab}>--------{type(o).__name__} class instance\n')
        for name, val in vars(o).items():
            if hasattr(val, '__dataclass_fields__'):
                lines(val, f, n + 1)
            else:
                f.write(f'{tab} - {name} = {val}\n')
        f.write(f'{tab}_______\n')
    with open(f'{foldername}/{type(obj).__name__}_text.txt', 'w') as f:
        lines(obj, f)
