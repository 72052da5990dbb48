"""Reader for the RTD1 named-array container written by oracle/rtdump.h (test infrastructure)."""
import struct

import numpy as np

_DT = {ord("f"): np.float32, ord("d"): np.float64, ord("i"): np.int32, ord("I"): np.uint32,
       ord("q"): np.int64, ord("Q"): np.uint64, ord("B"): np.uint8}


def load(path):
    out = {}
    with open(path, "rb") as f:
        if f.read(4) != b"RTD1":
            raise ValueError(f"{path}: not an RTD1 file")
        while True:
            (n,) = struct.unpack("<I", f.read(4))
            if n == 0:
                break
            name = f.read(n).decode()
            dt, nd = struct.unpack("<BB", f.read(2))
            shape = struct.unpack("<%dQ" % nd, f.read(8 * nd))
            dtype = np.dtype(_DT[dt])
            count = int(np.prod(shape)) if shape else 1
            out[name] = np.frombuffer(f.read(count * dtype.itemsize), dtype=dtype).reshape(shape)
    return out


def save(path, arrays):
    codes = {np.dtype(v): k for k, v in _DT.items()}
    with open(path, "wb") as f:
        f.write(b"RTD1")
        for name, a in arrays.items():
            a = np.ascontiguousarray(a)
            nb = name.encode()
            f.write(struct.pack("<I", len(nb)) + nb)
            f.write(struct.pack("<BB", codes[a.dtype], a.ndim))
            f.write(struct.pack("<%dQ" % a.ndim, *a.shape))
            f.write(a.tobytes())
        f.write(struct.pack("<I", 0))
