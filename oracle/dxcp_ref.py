"""TEST INFRASTRUCTURE ONLY -- float64 CPU restatement of the reference's
DXCP-PhaT sampling-rate-offset estimator (``dxcpphat/sro_estimation.py:
180-345``, class ``DXCPPhaT``, default parameters) used as the parity checker
of the device estimator (``danse_amd/dxcp.py``).  Pinned against the
reference's own outputs on seeded two-channel signals
(``tests/golden/dxcp_*.npz``, ``tests/test_oracle_golden.py``).

Same NumPy / SciPy calls in the same order as the reference; the only
difference is storage (no debug fields).  Quirk kept: the zeroing of the
incoherent bins of the averaged CSD-2 writes into the running average itself
(``GCSD2_avg_ifft = self.GCSD2_avg`` aliases, sro_estimation.py:267-272).
"""
from __future__ import annotations

import math

import numpy as np
from scipy import signal

FS = 16000
FRAME = 2048          # FrameSize_input = FFTshift_dxcp
NFFT = 2 ** 13        # FFTsize_dxcp


class DXCPPhaT:
    """``DXCPPhaT`` with the reference's default parameters
    (``sro_estimation.py:130-145``)."""

    def __init__(self):
        self.fs = FS
        self.FrameSize_input = FRAME
        self.FFTshift_dxcp = FRAME
        self.FFTsize_dxcp = NFFT
        self.AccumTime_B_sec = 5
        self.SmoConst_CSDPhaT_alpha = .53
        self.SmoConst_CSDPhaT_alpha2 = .99
        self.SmoConst_SSOest_alpha = .99
        self.AddContWait_NumFr = 0
        self.SettlingCSD2avg_NumFr = 4
        self.X_12_abs_min = 1e-12
        self.SROmax_abs_ppm = 1000
        self.p_upsmpFac = 4
        # implicit parameters (sro_estimation.py:198-215)
        self.LowFreq_InpSig_fl_Hz = .01 * self.fs / 2
        self.UppFreq_InpSig_fu_Hz = .95 * self.fs / 2
        self.RateDXCPPhaT_Hz = self.fs / self.FFTshift_dxcp
        self.AccumTime_B_NumFr = int(self.AccumTime_B_sec // (1 / self.RateDXCPPhaT_Hz))
        self.B_smpls = self.AccumTime_B_NumFr * self.FFTshift_dxcp
        self.Upsilon = int(self.FFTsize_dxcp / 2 - 1)
        self.Lambda = int(((self.B_smpls * self.SROmax_abs_ppm) // 1e6) + 1)
        self.Cont_NumFr = self.AccumTime_B_NumFr + 1
        self.InvShiftFactor_NumFr = int(self.FFTsize_dxcp / self.FFTshift_dxcp)
        self.FFT_Nyq = int(self.FFTsize_dxcp / 2 + 1)
        self.FreqResol = self.fs / self.FFTsize_dxcp
        self.LowFreq_InpSig_fl_bin = int(self.LowFreq_InpSig_fl_Hz // self.FreqResol)
        self.UppFreq_InpSig_fu_bin = int(self.UppFreq_InpSig_fu_Hz // self.FreqResol)
        self.NyqDist_fu_bin = self.FFT_Nyq - self.UppFreq_InpSig_fu_bin
        # state
        self.SROppm_est_ell = 0
        self.SSOsmp_est_ell = 0
        self.GCSD_PhaT_avg = np.zeros((NFFT, 1), dtype=complex)
        self.GCSD_PhaT_avg_Cont = np.zeros((NFFT, self.Cont_NumFr), dtype=complex)
        self.GCSD2_avg = np.zeros((NFFT, 1), dtype=complex)
        self.GCCF1_smShftAvg = np.zeros((2 * self.Upsilon + 1, 1), dtype=float)
        self.InputBuffer = np.zeros((NFFT, 2), dtype=float)
        self.flag_initiated = False
        self.ell_execDXCPPhaT = 1
        self.ell = 1

    def _zero_incoherent(self, x):
        """sro_estimation.py:269-272 / 320-323 (in place)."""
        x[np.arange(self.LowFreq_InpSig_fl_bin)] = 0
        x[np.arange(NFFT - self.LowFreq_InpSig_fl_bin + 1, NFFT)] = 0
        x[np.arange(self.FFT_Nyq - self.NyqDist_fu_bin - 1, self.FFT_Nyq + self.NyqDist_fu_bin)] = 0

    def process_data(self, x_12_ell):
        """``process_data`` (sro_estimation.py:218-238): x_12_ell (2048, 2)."""
        self.InputBuffer[:NFFT - FRAME, :] = self.InputBuffer[FRAME:, :]
        self.InputBuffer[NFFT - FRAME:, :] = x_12_ell
        if self.ell_execDXCPPhaT == int(self.FFTshift_dxcp / self.FrameSize_input):
            self.ell_execDXCPPhaT = 0
            self._stateupdate()
        self.ell_execDXCPPhaT += 1
        return {'SROppm_est_out': self.SROppm_est_ell, 'STOsmp_est_out': self.SSOsmp_est_ell}

    def _stateupdate(self):
        """``_stateupdate`` (sro_estimation.py:241-345), tdoa = 0."""
        analWin = signal.windows.blackman(NFFT, sym=False)
        x_12_win = self.InputBuffer * np.vstack((analWin, analWin)).transpose()
        X_12 = np.fft.fft(x_12_win, NFFT, 0)
        X_12_act = X_12[:, 0] * np.conj(X_12[:, 1])
        X_12_act_abs = abs(X_12_act)
        X_12_act_abs[X_12_act_abs < self.X_12_abs_min] = self.X_12_abs_min
        GCSD_PhaT_act = X_12_act / X_12_act_abs
        if not self.flag_initiated:
            self.GCSD_PhaT_avg = GCSD_PhaT_act
        else:
            a = self.SmoConst_CSDPhaT_alpha
            self.GCSD_PhaT_avg = a * self.GCSD_PhaT_avg + (1 - a) * GCSD_PhaT_act
        self.GCSD_PhaT_avg_Cont[:, np.arange(self.Cont_NumFr - 1)] = self.GCSD_PhaT_avg_Cont[:, 1:]
        self.GCSD_PhaT_avg_Cont[:, self.Cont_NumFr - 1] = self.GCSD_PhaT_avg
        start = self.Cont_NumFr + (self.InvShiftFactor_NumFr - 1) + self.AddContWait_NumFr
        if self.ell >= start:
            GCSD2_act = self.GCSD_PhaT_avg_Cont[:, -1] * np.conj(self.GCSD_PhaT_avg_Cont[:, 0])
            if not self.flag_initiated:
                self.GCSD2_avg[:, 0] = GCSD2_act
            else:
                a2 = self.SmoConst_CSDPhaT_alpha2
                self.GCSD2_avg[:, 0] = a2 * self.GCSD2_avg[:, 0] + (1 - a2) * GCSD2_act
            GCSD2_avg_ifft = self.GCSD2_avg          # aliases the running average (quirk)
            self._zero_incoherent(GCSD2_avg_ifft[:, 0])
            big = np.fft.fftshift(np.real(np.fft.ifft(GCSD2_avg_ifft, n=NFFT, axis=0)))
            idx = np.arange(self.FFT_Nyq - self.Lambda - 1, self.FFT_Nyq + self.Lambda)
            self.GCCF2avg_ell = big[idx, 0]
        if self.ell >= start + self.SettlingCSD2avg_NumFr:
            upsmpWindow = signal.get_window(('kaiser', 5.0), Nx=2 * self.Lambda + 1, fftbins=False)
            up = signal.resample(self.GCCF2avg_ell, num=(2 * self.Lambda + 1) * self.p_upsmpFac, window=upsmpWindow)
            lam = np.arange(-self.Lambda, self.Lambda + 1, 1 / self.p_upsmpFac)
            im = up.argmax(0)
            if im == 0 or im == len(lam) - 1:
                frac = 0
            else:
                sp = up[np.arange(im - 1, im + 2)]
                frac = (sp[2] - sp[0]) / 2 / (2 * sp[1] - sp[2] - sp[0])
            self.SROppm_est_ell = (lam[im] + frac / self.p_upsmpFac) / self.B_smpls * 10 ** 6
            # STO after removing the SRO-induced time offset in CCF-1
            timeOffset = self.SROppm_est_ell * 10 ** (-6) * self.FFTshift_dxcp * (self.ell - 1)
            k = np.arange(NFFT).transpose()
            expTerm = np.power(math.e, 1j * 2 * math.pi / NFFT * timeOffset * k)
            G1 = self.GCSD_PhaT_avg * expTerm
            self._zero_incoherent(G1)
            big1 = np.fft.fftshift(np.real(np.fft.ifft(G1, n=NFFT)))
            cc1 = big1[np.arange(self.FFT_Nyq - self.Upsilon - 1, self.FFT_Nyq + self.Upsilon)]
            if not self.flag_initiated:
                self.GCCF1_smShftAvg[:, 0] = cc1
            else:
                a3 = self.SmoConst_SSOest_alpha
                self.GCCF1_smShftAvg[:, 0] = a3 * self.GCCF1_smShftAvg[:, 0] + (1 - a3) * cc1
            ab = np.abs(self.GCCF1_smShftAvg)
            im1 = ab.argmax(0)
            if im1 == 0 or im1 == 2 * self.Upsilon:
                self.SSOsmp_est_ell = im1[0] - self.Upsilon
            else:
                sp = ab[np.arange(im1 - 1, im1 + 2)]
                fr = (sp[2] - sp[0]) / 2 / (2 * sp[1] - sp[2] - sp[0])
                self.SSOsmp_est_ell = im1[0] - self.Upsilon + fr[0]
        self.ell += 1
        if not self.flag_initiated:
            self.flag_initiated = True


def run(x1, x2):
    """Feed two channels frame by frame; per-frame (SRO ppm, STO samples)."""
    est = DXCPPhaT()
    n = len(x1) // FRAME
    sro = np.zeros(n)
    sto = np.zeros(n)
    for i in range(n):
        fr = np.stack((x1[i * FRAME:(i + 1) * FRAME], x2[i * FRAME:(i + 1) * FRAME]), axis=1)
        out = est.process_data(fr)
        sro[i] = out['SROppm_est_out']
        sto[i] = out['STOsmp_est_out']
    return sro, sto


# --------------------------------------------------------------------------- #
# Closed loop: CL_DXCPPhaT (sro_estimation.py:12-72) with its
# OnlineResampler (online_resampler.py:4-77) and DelayBuffer
# (delay_buffer.py:8-26); the same NumPy calls in the same order.
# --------------------------------------------------------------------------- #
class DelayBuffer:
    def __init__(self, shape):
        self.data = np.zeros(shape)
        self.length = shape[-1]
        self.pointer = 0

    def write(self, frame):
        self.data[..., self.pointer] = frame
        self.pointer = (self.pointer + 1) % self.length

    def read(self):
        return self.data[..., self.pointer]


class OnlineResampler:
    """Integer shift by buffer selection, fractional rest by a linear phase
    on the 2x-interpolated FFT of the Hann-windowed two-block selection,
    overlap-added: returns the block from two calls earlier."""

    def __init__(self, blockSize=FRAME):
        self.blockSize = blockSize
        self.fftSize = blockSize * 4
        self.shift = 0
        self.k = np.fft.fftshift(np.arange(-self.fftSize / 2, self.fftSize / 2))
        self.win = signal.windows.hann(blockSize * 2, sym=False)
        self.inputBuffer = np.zeros((blockSize * 4,))
        self.outputBuffer = np.zeros((blockSize * 3,))

    def process(self, signalBlock, sro, sto=0):
        B = self.blockSize
        self.inputBuffer[:(3 * B)] = self.inputBuffer[B:]
        self.inputBuffer[3 * B:] = signalBlock
        self.shift += sro * 1e-6 * B
        accShift = self.shift + sto
        integer_shift = np.round(accShift)
        rest_shift = integer_shift - accShift
        selectStart = int(B + integer_shift)
        selectEnd = int((B + 2 * B) + integer_shift)
        if selectStart < 0:
            self.shift -= sro * 1e-6 * B
            selectEnd = selectEnd - selectStart
            selectStart = 0
        elif selectEnd >= np.size(self.inputBuffer):
            self.shift -= sro * 1e-6 * B
            selectStart = selectStart - (selectEnd - np.size(self.inputBuffer))
            selectEnd = np.size(self.inputBuffer)
        sel = self.inputBuffer[selectStart:selectEnd]
        X = np.fft.fft(self.win * sel, self.fftSize)
        X *= np.exp(-1j * 2 * np.pi * self.k / self.fftSize * rest_shift)
        self.outputBuffer[B:] = self.outputBuffer[B:] + np.real(np.fft.ifft(X))[:int(B * 2)]
        self.outputBuffer[:2 * B] = self.outputBuffer[B:]
        self.outputBuffer[2 * B:] = np.zeros((B,))
        return self.outputBuffer[:B]


class CL_DXCPPhaT:
    """Resample z_i with the current estimate, delay z_j by the resampler's
    two blocks (+1), DXCP-PhaT on the synchronised pair, IMC controller
    (PIT1, Tf = 8) on the residual."""

    def __init__(self, start_delay=0):
        self.DXCPPhaT = DXCPPhaT()
        self.Resampler = OnlineResampler()
        self.zjBuffer = DelayBuffer((FRAME, 2 + 1))
        self.dSRO_est = np.zeros(3)
        self.SRO_est = np.zeros(3)
        self.dSRO_est_curr = 0
        self.dSRO_est_curr_raw = 0
        self.SRO_est_curr = 0
        self.SRO_est_op = 0
        self.K_Nom = [0, 0.0251941968627353, -0.0249422548941180]
        self.K_Denom = [1, -1.96825464010938, 0.968254640109407]
        self.start_delay = start_delay
        self.ell = 0

    def process(self, x_12_ell, acs=1):
        x_12_ell = np.array(x_12_ell, dtype=np.float64)
        z_i = self.Resampler.process(x_12_ell[:, 1].flatten(), -self.SRO_est_curr)
        x_12_ell[:, 1] = z_i
        self.zjBuffer.write(x_12_ell[:, 0].flatten())
        x_12_ell[:, 0] = self.zjBuffer.read()
        res = self.DXCPPhaT.process_data(x_12_ell)
        self.dSRO_est_curr_raw = res['SROppm_est_out']
        self.dSRO_est_curr = res['SROppm_est_out'] if acs == 1 else 0
        if self.ell <= self.start_delay:
            self.dSRO_est_curr = 0
        self.dSRO_est[1:] = self.dSRO_est[:-1]
        self.dSRO_est[0] = self.dSRO_est_curr
        self.SRO_est[1:] = self.SRO_est[:-1]
        self.SRO_est[0] = np.dot(self.K_Nom, self.dSRO_est) - np.dot(self.K_Denom[1:], self.SRO_est[1:])
        self.SRO_est_curr = self.SRO_est[0] + self.SRO_est_op
        self.ell += 1
        return self.dSRO_est_curr_raw, self.SRO_est_curr, self.Resampler.shift, z_i


def run_closed_loop(x1, x2, start_delay=0, acs=None):
    """Feed (z_j = x1, z_i = x2) frame by frame; per frame (raw residual ppm,
    controlled SRO estimate ppm, resampler shift, synchronised z_i block)."""
    cl = CL_DXCPPhaT(start_delay)
    n = len(x1) // FRAME
    out = np.zeros((n, 3))
    zi = np.zeros((n, FRAME))
    for i in range(n):
        fr = np.stack((x1[i * FRAME:(i + 1) * FRAME], x2[i * FRAME:(i + 1) * FRAME]), axis=1)
        a = 1 if acs is None else int(acs[i])
        d, s, sh, z = cl.process(fr, a)
        out[i] = (d, s, sh)
        zi[i] = z
    return out, zi
