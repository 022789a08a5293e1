#!/usr/bin/env python3
"""Make the JPEG golden vectors in tests/golden/jpeg/ (run in the build container).

The reference's default mode runs PyTurboJPEG (inverter.py:32,44; webcam_app.py:110,140),
i.e. libturbojpeg from libjpeg-turbo.  Neither PyTurboJPEG nor libturbojpeg is installed,
but the image's libjpeg-turbo 2.1.2 (libjpeg.so.8, the codec libturbojpeg wraps) is; it is
driven the way TurboJPEG drives it by oracle/jpeg_xcheck.c.  Every vector below is produced
by that library, not by the oracle or the product:

  file              a JPEG encoded by libjpeg-turbo from a seeded synthetic frame
  decoded_sha256    libjpeg-turbo's decode of it (TJPF_BGR, fancy upsampling, islow IDCT)
  inverted_sha256   libjpeg-turbo's encode (q85, 4:2:2, islow) of ~decoded: the reference
                    InverterWorker output with use_jpeg=True (inverter.py:31-44)
  reencoded_sha256  libjpeg-turbo's encode (q85, 4:2:2, islow) of decoded

    python tests/golden/make_jpeg_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import jpeg as J  # noqa: E402

OUT = os.path.join(HERE, "jpeg")

CASES = [  # (name, kind, seed, h, w, quality, subsamp, fastdct)
    ("scene_480p_q85_422", "scene", 0, 480, 640, 85, J.TJSAMP_422, False),
    ("scene_480p_q75_420", "scene", 1, 480, 640, 75, J.TJSAMP_420, False),
    ("scene_270x360_q90_444_fast", "scene", 2, 270, 360, 90, J.TJSAMP_444, True),
    ("scene_120x160_q85_gray", "scene", 3, 120, 160, 85, J.TJSAMP_GRAY, False),
    ("scene_96x128_q60_440", "scene", 4, 96, 128, 60, J.TJSAMP_440, False),
    ("scene_17x13_q85_422", "scene", 5, 17, 13, 85, J.TJSAMP_422, False),
    ("scene_33x9_q85_420", "scene", 6, 33, 9, 85, J.TJSAMP_420, False),
    ("noise_64x48_q85_422", "noise", 7, 64, 48, 85, J.TJSAMP_422, False),
    ("noise_16x16_q100_444", "noise", 8, 16, 16, 100, J.TJSAMP_444, False),
    ("flat_1x1_q85_422", "flat", 9, 1, 1, 85, J.TJSAMP_422, False),
    # libjpeg options TurboJPEG leaves off, which a decoder of arbitrary producers meets:
    # restart intervals (DRI + RSTn; per MCU count or per MCU row) and optimised Huffman tables
    ("scene_480p_q85_422_dri4", "scene", 10, 480, 640, 85, J.TJSAMP_422, False, {"restart_interval": 4}),
    ("scene_270x360_q85_420_drirow_opt", "scene", 11, 270, 360, 85, J.TJSAMP_420, False,
     {"restart_rows": 1, "optimize": True}),
    ("scene_120x160_q85_gray_dri1", "scene", 12, 120, 160, 85, J.TJSAMP_GRAY, False, {"restart_interval": 1}),
    ("noise_64x48_q90_444_dri7_opt", "noise", 13, 64, 48, 90, J.TJSAMP_444, False,
     {"restart_interval": 7, "optimize": True}),
    ("scene_96x128_q75_440_opt", "scene", 14, 96, 128, 75, J.TJSAMP_440, False, {"optimize": True}),
    ("scene_33x9_q85_422_dri2", "scene", 15, 33, 9, 85, J.TJSAMP_422, False, {"restart_interval": 2}),
    # the reference app's own operating point: webcam_app.py:17,97-111 centre-crops to 512 x 512
    # and encodes with PyTurboJPEG's defaults (q85, 4:2:2)
    ("scene_512sq_q85_422", "scene", 16, 512, 512, 85, J.TJSAMP_422, False),
    ("noise_512sq_q85_422", "noise", 17, 512, 512, 85, J.TJSAMP_422, False),
]


def frame(kind, seed, h, w):
    if kind == "noise":
        return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)
    if kind == "flat":
        return np.full((h, w, 3), 200, np.uint8)
    return J.synthetic_scene(seed, h, w)


def main():
    ok, why = J.libjpeg_available()
    if not ok:
        sys.exit(f"libjpeg-turbo not usable: {why}")
    os.makedirs(OUT, exist_ok=True)
    cases = []
    for name, kind, seed, h, w, q, ss, fast, *opt in CASES:
        opt = opt[0] if opt else {}
        img = frame(kind, seed, h, w)
        jpg = J.libjpeg_encode(img, q, J.TJPF_BGR, ss, fast, **opt)
        dec = J.libjpeg_decode(jpg, J.TJPF_BGR)
        inv = J.libjpeg_encode(np.bitwise_not(dec), 85, J.TJPF_BGR, J.TJSAMP_422, False)
        rec = J.libjpeg_encode(dec, 85, J.TJPF_BGR, J.TJSAMP_422, False)
        fn = name + ".jpg"
        with open(os.path.join(OUT, fn), "wb") as f:
            f.write(jpg)
        cases.append({
            "file": fn, "kind": kind, "seed": seed, "shape": [h, w, 3], "quality": q, "subsamp": ss,
            "fastdct": fast, "libjpeg_options": opt,
            "source_sha256": hashlib.sha256(img.tobytes()).hexdigest(),
            "jpeg_sha256": hashlib.sha256(jpg).hexdigest(),
            "decoded_sha256": hashlib.sha256(dec.tobytes()).hexdigest(),
            "inverted_sha256": hashlib.sha256(inv).hexdigest(),
            "reencoded_sha256": hashlib.sha256(rec).hexdigest(),
        })
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump({"generator": "libjpeg-turbo 2.1.2 (libjpeg.so.8) via oracle/jpeg_xcheck.c; "
                                "tests/golden/make_jpeg_golden.py", "libjpeg": why, "cases": cases}, f, indent=1)
    print(f"wrote {len(cases)} cases to {OUT}")


if __name__ == "__main__":
    main()
