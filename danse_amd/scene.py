"""Synthetic acoustic scenes for the DANSE engine (input producer).

Scene generation is not on the hot path; this module exists so that tests, the
oracle and ``bench.py`` all feed the engine bit-identical inputs from a seed.
It follows the *shape* of the reference's offline scene path
(``trueRoom: false``, ``signalType: random``):

* random impulse responses, uniform in [-0.5, 0.5], 0.2 s, no decay
  (``siggen/utils.py:229-308``, ``siggen/classes.py:16-29``);
* uniform [-1, 1] desired source with predefined 0.5 s pauses every 0.5 s, and
  one continuous uniform noise source (``siggen/classes.py:32-64``);
* SNR set at mic 0 (``siggen/utils.py:1421-1431``) and white self-noise per
  sensor (``siggen/utils.py:1418``);
* an energy VAD on the wet desired signal at each node's reference sensor
  (``siggen/utils.py:834-939,1079-1133``).

It is NOT a bit-exact restatement of ``siggen`` (different RNG streams, a
vectorised VAD): parity is anchored by injecting the very same arrays into the
reference, the oracle and the GPU engine.  All signals are rounded to float32
(and kept as float64 values) so that the fp32 device path and the fp64 oracle
consume exactly the same numbers.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
from scipy.signal import fftconvolve


@dataclass
class SceneNode:
    """The fields of ``siggen.classes.Node`` (``siggen/classes.py:379-428``)
    that the DANSE engine reads."""
    index: int
    nSensors: int
    fs: float
    data: np.ndarray            # [T x M] noisy mic signals
    cleanspeech: np.ndarray     # [T x M] speech-only
    cleannoise: np.ndarray      # [T x M] noise-only (incl. ref-sensor self-noise)
    timeStamps: np.ndarray      # [T]
    vad: np.ndarray             # [T x 1] per-sample VAD (0/1)
    neighborsIdx: list = field(default_factory=list)
    sro: float = 0.0
    refSensorIdx: int = 0
    vadPerFrame: np.ndarray = None
    beta: float = 1.0
    betaWext: float = 1.0


@dataclass
class Scene:
    """A fully connected WASN (``siggen.classes.WASN``, ``siggen/classes.py:431``)."""
    wasn: list
    fs: float
    seed: int

    @property
    def nNodes(self) -> int:
        return len(self.wasn)

    @property
    def nSensorPerNode(self) -> list:
        return [n.nSensors for n in self.wasn]

    def get_vad_per_frame(self, frameLen: int, frameShift: int, minProportionActive: float = 0.5):
        """Frame VAD, restating ``WASN.get_vad_per_frame``
        (``siggen/classes.py:669-702``), including its crop quirk: when the
        frame running past the end is met at index ``ii``, the output keeps
        ``ii + 1`` entries (the last one stays 0)."""
        for node in self.wasn:
            node.vadPerFrame = vad_per_frame(node.vad[:, 0], frameLen, frameShift, minProportionActive)


def vad_per_frame(vad: np.ndarray, frameLen: int, frameShift: int, minProp: float) -> np.ndarray:
    n = len(vad)
    nFrames = n // frameShift
    out = np.zeros(nFrames, dtype=bool)
    csum = np.concatenate(([0.0], np.cumsum(vad, dtype=np.float64)))
    for ii in range(nFrames):
        b, e = ii * frameShift, ii * frameShift + frameLen
        if e > n:
            return out[:ii + 1]
        out[ii] = (csum[e] - csum[b]) >= frameLen * minProp
    return out


def _energy_vad(x: np.ndarray, fs: float, tw: float, energyDecrease_dB: float) -> np.ndarray:
    """Short-time energy VAD: window of ``int(tw*fs)`` samples centred on each
    sample, active if the window energy exceeds max(x^2)/10^(dB/10)
    (shape of ``oracleVAD``, ``siggen/utils.py:1079-1133``)."""
    thrs = np.amax(x ** 2) / (10 ** (energyDecrease_dB / 10))
    nw = max(int(tw * fs), 1)
    c = np.concatenate(([0.0], np.cumsum(x ** 2)))
    idx = np.arange(len(x))
    b = np.maximum(idx - nw // 2, 0)
    e = np.minimum(idx + nw // 2, len(x))
    energy = c[e] - c[b]
    return (energy > thrs).astype(np.float64)


def _f32(x: np.ndarray) -> np.ndarray:
    return np.asarray(x, dtype=np.float32).astype(np.float64)


def make_scene(
    nSensorPerNode,
    sigDur: float = 10.0,
    fs: float = 16000.0,
    seed: int = 0,
    snr: float = 5.0,
    selfnoiseSNR: float = 15.0,
    irDuration: float = 0.2,
    pauseDuration: float = 0.5,
    pauseSpacing: float = 0.5,
    vadEnergyDecrease_dB: float = 40.0,
    vadWinLength: float = 0.04,
    SROperNode=None,
    nodes=None,
) -> Scene:
    """Build a random-IR, random-signal fully connected WASN.

    Every node draws from its own RNG stream (``default_rng([seed, 1, k])``),
    the two sources from ``default_rng([seed, 0])``, so any subset of nodes
    can be generated on its own (``nodes``; multi-GPU ranks build only the
    nodes they own).  Nodes outside ``nodes`` get all-zero signals.  The noise
    gain that sets the SNR at mic 0 of node 0 always uses node 0.

    SROs are recorded per node (``SROperNode`` in ppm) but the signals are not
    resampled here (the reference needs ``resampy`` for that, absent offline);
    the time stamps follow ``siggen/utils.py:1579-1622`` (``t = n / fsSRO``).
    """
    K = len(nSensorPerNode)
    T = int(sigDur * fs)
    nIR = int(irDuration * fs)
    sros = np.zeros(K) if SROperNode is None else np.asarray(SROperNode, dtype=float)
    want = set(range(K)) if nodes is None else set(int(k) for k in nodes)

    src = np.random.default_rng([seed, 0])
    # Desired source: uniform noise with predefined pauses (0.5 s on / 0.5 s off).
    d = src.uniform(-1.0, 1.0, T)
    t = np.arange(T) / fs
    period = pauseDuration + pauseSpacing
    d[(t % period) >= pauseSpacing] = 0.0
    n = src.uniform(-1.0, 1.0, T)

    def wet(k):
        rng = np.random.default_rng([seed, 1, k])
        M = int(nSensorPerNode[k])
        wS = np.zeros((T, M))
        wN = np.zeros((T, M))
        for m in range(M):
            wS[:, m] = fftconvolve(d, rng.uniform(-0.5, 0.5, nIR))[:T]
            wN[:, m] = fftconvolve(n, rng.uniform(-0.5, 0.5, nIR))[:T]
        return rng, wS, wN

    rng0, wS0, wN0 = wet(0)
    # SNR at mic 0 of node 0 (single noise source).
    Ps = np.mean(wS0[:, 0] ** 2)
    Pn = np.mean(wN0[:, 0] ** 2)
    gN = 10 ** (-(snr - 10 * np.log10(Ps / Pn)) / 20)

    wasn = []
    for k in range(K):
        M = int(nSensorPerNode[k])
        fsSRO = fs * (1 + sros[k] / 1e6)
        common = dict(index=k, nSensors=M, fs=fsSRO, timeStamps=np.arange(T) / fsSRO,
                      neighborsIdx=[q for q in range(K) if q != k], sro=float(sros[k]))
        if k not in want:
            z = np.zeros((T, M))
            wasn.append(SceneNode(data=z, cleanspeech=z, cleannoise=z, vad=np.zeros((T, 1)), **common))
            continue
        rng, wS, wN = (rng0, wS0, wN0) if k == 0 else wet(k)
        wN = wN * gN
        clean = wS + wN
        sig = np.zeros_like(clean)
        selfN = np.zeros_like(clean)
        for m in range(M):
            sn = rng.uniform(-1.0, 1.0, T)
            Pc = np.mean(clean[:, m] ** 2)
            Psn = np.mean(sn ** 2)
            sn *= 10 ** (-(selfnoiseSNR - 10 * np.log10(Pc / Psn)) / 20)
            selfN[:, m] = sn
            sig[:, m] = clean[:, m] + sn
        vad = _energy_vad(wS[:, 0], fs, vadWinLength, vadEnergyDecrease_dB)
        wasn.append(SceneNode(data=_f32(sig), cleanspeech=_f32(wS), cleannoise=_f32(wN + selfN[:, :1]),
                              vad=vad[:, None], **common))
    return Scene(wasn=wasn, fs=fs, seed=seed)


def scene_digest(scene: Scene) -> str:
    """sha256 over the float32 input bytes: pins that a scene regenerated from
    its seed on another machine is the one the golden fixtures were made on."""
    import hashlib
    h = hashlib.sha256()
    for node in scene.wasn:
        h.update(node.data.astype(np.float32).tobytes())
        h.update(node.vad.astype(np.uint8).tobytes())
    return h.hexdigest()


def make_scenes_device(nSensorPerNode, S, sigDur=10.0, fs=16000.0, seed=0, snr=5.0, selfnoiseSNR=15.0,
                       irDuration=0.2, pauseDuration=0.5, pauseSpacing=0.5, vadEnergyDecrease_dB=40.0,
                       vadWinLength=0.04, SROperNode=None, device=0, host_signals=False):
    """S random-IR scenes generated on the device (``danse_scene_generate``,
    csrc/scene.hip): the same scene model as :func:`make_scene`, with its own
    counter-based random numbers (scene s from ``seed + s``) and the SRO
    resampling that :func:`make_scene` omits (node k's signals at
    fs (1 + SRO_k 1e-6); our Kaiser-windowed sinc, the reference uses
    resampy).  Returns ``(scenes, dev)``: Scene objects whose nodes carry the
    time stamps, VAD and -- with ``host_signals`` -- the signals as float32
    host arrays, and ``dev`` = dict of device tensors ``data``,
    ``cleanspeech``, ``cleannoise`` [S][sum M][T] float32 and ``vad``
    [S][K][T] uint8 (``DanseEngine(..., yDevice=dev['data'])`` takes the
    inputs without a host round trip)."""
    import ctypes
    import torch
    from . import _lib as L
    lib = L.load_library()
    M = [int(m) for m in nSensorPerNode]
    K, MT, T = len(M), int(sum(M)), int(sigDur * fs)
    dev = f'cuda:{device}'
    out = {key: torch.empty((S, MT, T), dtype=torch.float32, device=dev) for key in ('data', 'cleanspeech', 'cleannoise')}
    out['vad'] = torch.empty((S, K, T), dtype=torch.uint8, device=dev)
    sros = np.zeros(K) if SROperNode is None else np.asarray(SROperNode, dtype=np.float64)
    Marr = np.asarray(M, dtype=np.int32)
    sroArr = np.ascontiguousarray(sros, dtype=np.float64)
    c = L.SceneCfg()
    c.S, c.K, c.M, c.T, c.nIR, c.seed = S, K, Marr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), T, \
        int(irDuration * fs), int(seed)
    c.fs, c.snr, c.selfnoiseSNR = float(fs), float(snr), float(selfnoiseSNR)
    c.pauseDuration, c.pauseSpacing = float(pauseDuration), float(pauseSpacing)
    c.vadEnergyDecrease_dB, c.vadWinLength = float(vadEnergyDecrease_dB), float(vadWinLength)
    c.sroPpm = sroArr.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    st = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    rc = lib.danse_scene_generate(ctypes.byref(c), ctypes.c_void_p(out['data'].data_ptr()),
                                  ctypes.c_void_p(out['cleanspeech'].data_ptr()),
                                  ctypes.c_void_p(out['cleannoise'].data_ptr()), ctypes.c_void_p(out['vad'].data_ptr()),
                                  st)
    if rc != 0:
        raise L.DanseError((lib.danse_scene_last_error() or b'').decode() or f'error {rc}')
    vad = out['vad'].cpu().numpy()   # 0/1 (uint8 on the device; float64 per node, as make_scene)
    host = {key: out[key].cpu().numpy() for key in ('data', 'cleanspeech', 'cleannoise')} if host_signals else None
    base = np.concatenate(([0], np.cumsum(M)[:-1])).astype(int)
    scenes = []
    for s in range(S):
        wasn = []
        for k in range(K):
            fsSRO = fs * (1 + sros[k] / 1e6)
            sl = slice(base[k], base[k] + M[k])
            sig = {key: (host[key][s, sl].T if host is not None else None) for key in ('data', 'cleanspeech', 'cleannoise')}
            wasn.append(SceneNode(index=k, nSensors=M[k], fs=fsSRO, timeStamps=np.arange(T) / fsSRO,
                                  neighborsIdx=[q for q in range(K) if q != k], sro=float(sros[k]),
                                  vad=vad[s, k][:, None].astype(np.float64), **sig))
        scenes.append(Scene(wasn=wasn, fs=fs, seed=seed + s))
    return scenes, out


def convolve_vad(x, h, fs=16000.0, vadWinLength=0.04, vadEnergyDecrease_dB=40.0, vad=True, device=0):
    """The device generator's convolution and VAD kernels on given rows
    (``danse_scene_convolve_vad``): ``x`` [rows][T] and ``h`` [rows][nIR]
    (host arrays, rounded to float32) -> (out [rows][T] float32 = (x * h)
    [:T], vad [rows][T] uint8 = oracleVAD(out), or None).  The checks of the
    generator against the reference's get_vad on injected inputs use it."""
    import ctypes
    import torch
    from . import _lib as L
    lib = L.load_library()
    dev = f'cuda:{device}'
    xt = torch.as_tensor(np.ascontiguousarray(x, dtype=np.float32), device=dev)
    ht = torch.as_tensor(np.ascontiguousarray(h, dtype=np.float32), device=dev)
    rows, T = xt.shape
    out = torch.empty((rows, T), dtype=torch.float32, device=dev)
    v = torch.empty((rows, T), dtype=torch.uint8, device=dev) if vad else None
    st = torch.cuda.current_stream(device).cuda_stream
    rc = lib.danse_scene_convolve_vad(ctypes.c_void_p(xt.data_ptr()), ctypes.c_void_p(ht.data_ptr()), int(rows),
                                      int(T), int(ht.shape[1]), ctypes.c_void_p(out.data_ptr()), float(vadWinLength),
                                      float(fs), float(vadEnergyDecrease_dB),
                                      ctypes.c_void_p(v.data_ptr() if v is not None else 0), ctypes.c_void_p(st))
    if rc != 0:
        raise L.DanseError((lib.danse_scene_last_error() or b'').decode() or f'error {rc}')
    return out.cpu().numpy(), (v.cpu().numpy() if v is not None else None)
