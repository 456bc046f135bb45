"""The crafted exceptional fixture (tests/golden/p256_crafted.bin) is what its generator
(tests/golden/gen_crafted.py) makes, byte for byte, and its verdicts are the oracle's: every
crafted doubling is a valid signature, R = infinity is rejected (CPU only)."""
import json
import os

import numpy as np

import oracle
from conftest import GOLDEN


def test_crafted_fixture_regenerates():
    import sys
    sys.path.insert(0, GOLDEN)
    import gen_crafted
    data, names = gen_crafted.records()
    assert data == open(os.path.join(GOLDEN, "p256_crafted.bin"), "rb").read()
    assert names == json.load(open(os.path.join(GOLDEN, "p256_crafted.json")))["tags"]


def test_crafted_fixture_verdicts():
    raw = np.fromfile(os.path.join(GOLDEN, "p256_crafted.bin"), dtype=np.uint8).reshape(-1, 162)
    names = json.load(open(os.path.join(GOLDEN, "p256_crafted.json")))["tags"]
    cols = [np.ascontiguousarray(raw[:, 32 * k:32 * k + 32]) for k in range(5)]
    assert np.array_equal(oracle.verify_batch(*cols), raw[:, 160])
    tags = [names[i] for i in raw[:, 161]]
    import sys
    sys.path.insert(0, GOLDEN)
    import gen_crafted
    # 16 ladder tuples + 3 x 2 x (K + 1) comb tuples (K = 12 windows of 22 bits), minus q = 0 / r = 0
    assert len(tags) > 80 and {t.rsplit("_", 1)[0] for t in tags} == {"ladder_last", "comb_dbl", "comb_inf"}
    for t, w in zip(tags, raw[:, 160]):
        if t.startswith(("comb_dbl", "ladder_last")):
            assert w == 1, t
        if t == f"comb_inf_{gen_crafted.KG}":  # the last step: R = infinity
            assert w == 0, t
