"""splitmix64 over numpy uint64 arrays (host-side twin of the device generator's hash)."""
import numpy as np

_C0 = np.uint64(0x9E3779B97F4A7C15)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)


def splitmix64_np(x):
    with np.errstate(over="ignore"):
        z = np.asarray(x, dtype=np.uint64) + _C0
        z = (z ^ (z >> np.uint64(30))) * _C1
        z = (z ^ (z >> np.uint64(27))) * _C2
        return z ^ (z >> np.uint64(31))
