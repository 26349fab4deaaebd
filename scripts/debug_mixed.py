import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import numpy as np
import p2p
from test_gpu_mixed import run_gpu, run_oracle, flows_grid
t0, period, count = [int(x) for x in sys.argv[1:4]]
sc = flows_grid()
app_send = [i for i, a in enumerate(sc.apps) if a["kind"] == p2p.APP_ONOFF][1]
app_obs = [i for i, a in enumerate(sc.apps) if a["kind"] == p2p.APP_SINK][0]
o = run_oracle(sc, t0, period, count, app_send, app_obs, 400000)
g = run_gpu(sc, t0, period, count, app_send, app_obs, 400000, 400000)
print("dispatched", g[0]["dispatched"], o[0].dispatched, "uid", g[0]["next_uid"], o[0].next_uid)
ol, gl = o[3], g[3]
n = int(o[0].dispatched)
for i in range(n):
    if ol[0][i] != gl[0][i] or ol[1][i] != gl[1][i]:
        print("first diff at", i)
        for j in range(max(0, i - 6), min(n, i + 6)):
            print(j, "oracle", int(ol[0][j]), int(ol[1][j]), int(ol[2][j]), "  gpu", int(gl[0][j]), int(gl[1][j]), int(gl[2][j]))
        break
else:
    print("logs equal")
print("samples equal", np.array_equal(o[5]["rx_packets"], g[5]["rx_packets"]))
