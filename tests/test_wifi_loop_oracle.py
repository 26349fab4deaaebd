"""The closed-loop Wi-Fi oracle (nsref_wifil_run) on the CPU: the error-rate models against their formulas
(nist-error-rate-model.cc, yans-error-rate-model.cc, dsss-error-rate-model.cc — restated here in Python from
the same lines), CalculatePer on an isolated reception (interference-helper.cc:257-334: the preamble is not a
chunk, the header at the header mode, the payload at the payload mode), and the run's invariants.  No
reference fixture pins SNR / PER (parity unpinned); tests/test_gpu_wifi_loop.py compares the device with this."""
import math

import numpy as np

import nsref
import wifi
from wifi_loop_harness import run_oracle, scenario


def test_dsss_and_nist_chunk_formulas():
    for snr in (0.05, 0.3, 1.0, 3.0, 8.0):
        for nbits in (1, 48, 1600):
            ber = 0.5 * math.exp(-snr * 22.0)  # GetDsssDbpskSuccessRate
            assert math.isclose(nsref.wifil_chunk_success(wifi.NIST, wifi.DSSS_1M, snr, nbits), (1 - ber) ** nbits,
                                rel_tol=1e-14)
            ber = 0.5 * math.erfc(math.sqrt(snr))  # Nist GetBpskBer, b = 1 (OFDM 6 Mb/s)
            D = math.sqrt(4.0 * ber * (1.0 - ber))
            pe = 0.5 * sum(c * D ** e for c, e in ((36.0, 10), (211.0, 12), (1404.0, 14), (11633.0, 16), (77433.0, 18),
                                                    (502690.0, 20), (3322763.0, 22), (21292910.0, 24),
                                                    (134365911.0, 26)))
            want = 1.0 if ber == 0.0 else (1 - min(pe, 1.0)) ** nbits
            got = nsref.wifil_chunk_success(wifi.NIST, (wifi.OFDM, 6000000, 20000000), snr, nbits)
            assert math.isclose(got, want, rel_tol=1e-12), (snr, nbits, got, want)


def test_yans_bpsk_chunk():
    snr, nbits = 0.7, 96
    mode = (wifi.OFDM, 6000000, 20000000)  # BPSK 1/2: phyRate 12 Mb/s, dFree 10, adFree 11
    ber = 0.5 * math.erfc(math.sqrt(snr * 20e6 / 12e6))
    fact = math.factorial
    pd = sum(fact(10) // (fact(i) * fact(10 - i)) * ber ** i * (1 - ber) ** (10 - i) for i in range(6, 10))
    pd += 0.5 * fact(10) // (fact(5) * fact(5)) * ber ** 5 * (1 - ber) ** 5
    want = (1 - min(11 * pd, 1.0)) ** nbits
    assert math.isclose(nsref.wifil_chunk_success(wifi.YANS, mode, snr, nbits), want, rel_tol=1e-12)


def test_isolated_reception_per():
    """Two phys 100 m apart, one SendPacket, nothing else on the air: PER = 1 - (header chunk at 1 Mb/s over
    48 us) x (payload chunk over the payload), SNR = P / (NF k T B)."""
    ph = wifi.LoopPhys(np.array([0.0, 100.0]), np.zeros(2), np.zeros(2))
    sc = dict(phys=ph, first=np.array([1000, 10 ** 9], np.uint64), backoff=np.array([10 ** 9, 10 ** 9], np.uint64),
              period=10 ** 9, stop_ns=50_000_000, size=200, mode=wifi.DSSS_1M, preamble=wifi.PREAMBLE_LONG,
              dbm=17.0206)
    log, ends, phys, tot = run_oracle(sc)
    assert tot["sends"] == 1 and len(ends) == 1 and phys["sync"][1] == 1
    rx_dbm = 17.0206 - (46.6777 + 30.0 * math.log10(100.0)) + 1.0
    w = 10 ** (rx_dbm / 10) / 1000
    snr = w / (10 ** 0.7 * 1.3803e-23 * 290.0 * 22e6)
    assert math.isclose(ends["snr"][0], snr, rel_tol=1e-12)
    pay_us = math.ceil(200 * 8 / 1.0)
    psr = (1 - 0.5 * math.exp(-snr * 22.0)) ** 48 * (1 - 0.5 * math.exp(-snr * 22.0)) ** pay_us
    assert math.isclose(ends["per"][0], 1 - psr, rel_tol=1e-9, abs_tol=1e-15)


def test_loop_invariants():
    sc = scenario()
    (lts, luid, lctx), ends, phys, tot = run_oracle(sc)
    assert tot["dispatched"] == len(lts)
    key = lts.astype(object) * (1 << 32) + luid
    assert all(key[i] < key[i + 1] for i in range(len(key) - 1))  # (ts, uid) order, each event once
    assert phys["end"].sum() == len(ends) and (phys["sync"] >= phys["end"]).all()
    assert phys["rx"].sum() <= tot["sends"] * (sc["phys"].n_phy - 1)  # (receptions after the Stop stay pending)
    assert (phys["rx"] == phys["sync"] + phys["drop_rx"] + phys["drop_tx"] + phys["drop_ed"]).all()
    assert ((ends["per"] >= 0) & (ends["per"] <= 1)).all()
