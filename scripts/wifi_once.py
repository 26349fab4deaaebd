"""One wifi-grid run (config 3 workload, Stop at argv[1] s) for rocprofv3 counter passes."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ns-3-dev-dnemu_amd"))
import nsgpu  # noqa: E402
import wifi  # noqa: E402

nsgpu.check(nsgpu.lib().nsgpu_set_device(0))
stop = float(sys.argv[1]) if len(sys.argv) > 1 else 0.5
eng = wifi.Engine(wifi.wifi_grid(n_side=100, stop_s=stop))
st = eng.run()
print("dispatched", st.dispatched, "store", eng.store())
eng.close()
