"""Diagnostic: k_wl_step per epoch at config-3 scale (lib/libnsgpu_prof.so): the slowest lane against the
average lane, and the events lanes run per epoch."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.argv = [sys.argv[0], "100", "1.0", "0.2", "0"]
sys.path[:0] = [os.path.join(REPO, "scripts")]
import numpy as np  # noqa: E402
exec(open(os.path.join(REPO, "scripts", "wifi_loop_scale.py")).read())
import nsgpu  # noqa: E402
buf = np.zeros(8, np.uint64)
nsgpu.check(nsgpu.lib().nsgpu_wifil_prof_read(buf.ctypes.data_as(C.c_void_p)))
ep = max(int(buf[5]), 1)
print(f"epochs {ep}: slowest lane {buf[0] * 10 / ep / 1e3:.1f} us/epoch, average lane {buf[1] * 10 / max(int(buf[2]), 1) / 1e3:.2f} us, "
      f"events per lane-epoch {buf[3] / max(int(buf[2]), 1):.2f}, most events one lane ran per epoch (mean) {buf[4] / ep:.1f}, "
      f"max lane {buf[6] * 10 / 1e3:.1f} us with {buf[7]} events")
