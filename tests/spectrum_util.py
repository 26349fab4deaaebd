"""Test helper: band edges of SpectrumModel (std::vector<double> centerFreqs) (spectrum-model.cc:44-72)."""
import numpy as np


def bands_from_centers(fc):
    fc = [float(v) for v in fc]
    fl, fh = [], []
    for i, c in enumerate(fc):
        if i == 0:
            d = (fc[1] - c) / 2
            fl.append(c - d)
            fh.append(c + d)
        elif i == len(fc) - 1:
            d = (c - fc[i - 1]) / 2
            fl.append(c - d)
            fh.append(c + d)
        else:
            fl.append((c + fc[i - 1]) / 2)
            fh.append((fc[i + 1] + c) / 2)
    return np.array(fl), np.array(fh)
