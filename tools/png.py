"""Tiny dependency-free PNG writer for viewing float images (gamma 1/2.2, clamp)."""
import struct
import sys
import zlib

import numpy as np


def write_png(path, img):
    a = np.asarray(img, dtype=np.float32)[..., :3]
    a = np.clip(np.nan_to_num(a), 0.0, 1.0) ** (1.0 / 2.2)
    a = (a * 255.0 + 0.5).astype(np.uint8)
    h, w, _ = a.shape
    raw = b"".join(b"\x00" + a[y].tobytes() for y in range(h))

    def chunk(t, d):
        c = struct.pack(">I", len(d)) + t + d
        return c + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw, 9)) + chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(png)


if __name__ == "__main__":
    write_png(sys.argv[2], np.load(sys.argv[1]))
