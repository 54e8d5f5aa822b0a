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
