"""Write the bench-simulator input distribution used by config 1.

utils/bench-simulator.cc:59-76 reads whitespace-separated doubles (seconds) and
converts each with (uint64_t)(data * 1000000000).  The survey fixes "10,000 initial
delays, uniform [0, 1) s" with a fixed seed; this script produces exactly that file
(shortest round-trip repr, so any strtod-compatible reader recovers the same doubles).
"""
import sys
import numpy as np

def main(path="tests/golden/bench_dist_u01_10k.txt", n=10000, seed=1):
    rng = np.random.Generator(np.random.PCG64(seed))
    vals = rng.random(n)
    with open(path, "w") as f:
        for v in vals:
            f.write(repr(float(v)) + "\n")

if __name__ == "__main__":
    main(*sys.argv[1:])
