"""Decode the reference's earth texture (assets/earthmap.jpg, used by EarthBuiltin,
image_texture.rs:11-20) once, into the raw RGB8 asset the host loads on the GPU box
(the reference tree does not travel there).  PIL decodes with libjpeg-turbo; the reference decodes
with jpeg-decoder 0.2.6 (Cargo.lock:525-526): texels may differ by <= 1 LSB (parity unpinned there).

usage: python tools/decode_earthmap.py /root/reference/assets/earthmap.jpg \
           shirley-raytracing-rs_amd/assets/earthmap.rgb8.gz
"""
import gzip
import sys

import numpy as np
from PIL import Image


def main(src, dst):
    a = np.asarray(Image.open(src).convert("RGB"))
    data = b"RGB8 %d %d\n" % (a.shape[1], a.shape[0]) + a.tobytes()
    open(dst, "wb").write(gzip.compress(data, 9, mtime=0))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
