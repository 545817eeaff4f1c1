"""Input-aware selector on the CPU: the matrix features
(GetInfo1/2/3), the density images and MatNet's forward pass in libias.so,
checked against
  * the reference's own printouts for Inputs/dia.mtx (features and "The Chosen
    One", CPU/1.jpg and GPU/2.jpg -> tests/golden/matnet_known_answers.json),
  * the oracle restatement (oracle/ias_oracle.c: ora_features,
    ora_density_image) on every sample input and synthetic matrices,
  * a float64 numpy restatement of MatNet.py Pred over the same weights (the
    library runs float32, as Keras does: probabilities within 1e-4),
  * the reference's .h5 weight files themselves when /root/reference is present
    (the committed blobs are their export, tools/matnet_export.py).
"""
import ctypes as C
import json
import os
import struct
import sys

import numpy as np
import pytest

import ias
import oracle_bind as ob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "ia-spgemm_amd", "data")
NAMES = ["dia.mtx", "small.mtx", "b1_ss.mtx", "Ragusa18.mtx", "LFAT5.mtx", "Trec5.mtx",
         "ch3-3-b2.mtx", "relat3.mtx", "sample.mtx"]
SETS = {"intel": (26, 5), "amd": (26, 5), "p100": (18, 3)}


def transpose(m):
    s, t = m.struct(), ias.Csr()
    ias.check(ias.lib.ias_csr_transpose(C.byref(s), C.byref(t)), "transpose")
    return ias.csr_to_numpy(t)


def synthetic():
    return [("rmat10", ias.gen_rmat(10, 8, seed=5)), ("band300", ias.gen_band(300, 2, seed=3)),
            ("ell128", ias.gen_ell(128, 5, seed=2))]


# ------------------------------------------------------------------ numpy MatNet (test restatement)
def load_blob(path):
    d = open(path, "rb").read()
    assert d[:8] == b"IASMNET1"
    nf, nc = struct.unpack_from("<ii", d, 8)
    conv = [(3, 3, 1, 16), (16,), (5, 5, 16, 16), (16,), (5, 5, 16, 16), (16,)]
    shapes = conv + conv + [(nf, nf), (nf,), (256, 32), (32,), (256, 32), (32,), (64 + nf, nc), (nc,)]
    off, w = 16, []
    for s in shapes:
        n = int(np.prod(s))
        w.append(np.frombuffer(d, "<f4", n, off).reshape(s).astype(np.float64))
        off += 4 * n
    assert off == len(d)
    return nf, nc, w


def np_conv(x, K, b, s, same):
    H, W, _ = x.shape
    k = K.shape[0]
    if same:
        OH, OW = -(-H // s), -(-W // s)
        ph, pw = max((OH - 1) * s + k - H, 0), max((OW - 1) * s + k - W, 0)
        x = np.pad(x, ((ph // 2, ph - ph // 2), (pw // 2, pw - pw // 2), (0, 0)))
    else:
        OH, OW = (H - k) // s + 1, (W - k) // s + 1
    out = np.zeros((OH, OW, K.shape[3]))
    for dy in range(k):
        for dx in range(k):
            out += x[dy:dy + s * (OH - 1) + 1:s, dx:dx + s * (OW - 1) + 1:s, :] @ K[dy, dx]
    return np.tanh(out + b)


def np_pool(x):
    H, W, Cc = x.shape
    return x[:H // 2 * 2, :W // 2 * 2].reshape(H // 2, 2, W // 2, 2, Cc).max(axis=(1, 3))


def np_matnet(blob, img_a, img_b, feats):
    """MatNet.py Pred (:29-92) in float64."""
    nf, nc, w = blob

    def branch(img, l):
        x = (img.astype(np.float64) * 255.0 / img.max()).reshape(128, 128, 1)
        x = np_pool(np_conv(x, w[2 * l], w[2 * l + 1], 1, False))
        x = np_pool(np_conv(x, w[2 * l + 2], w[2 * l + 3], 2, True))
        x = np_pool(np_conv(x, w[2 * l + 4], w[2 * l + 5], 2, True))
        return x.reshape(-1)

    a = np.tanh(branch(img_a, 0) @ w[14] + w[15])
    b = np.tanh(branch(img_b, 3) @ w[16] + w[17])
    f = np.tanh(np.asarray(feats, np.float64) @ w[12] + w[13])
    z = np.concatenate([a, b, f]) @ w[18] + w[19]
    p = np.exp(z - z.max())
    return p / p.sum()


# ------------------------------------------------------------------ tests
def test_known_answers_from_reference_printouts(inputs_dir, golden_dir):
    ka = json.load(open(os.path.join(golden_dir, "matnet_known_answers.json")))
    A, _ = ias.mtx_read(os.path.join(inputs_dir, "dia.mtx"))
    AT = transpose(A)
    for side in ("cpu", "gpu"):
        k = ka[side]
        f = ias.features(A, AT, k["nfeatures"])
        np.testing.assert_allclose(f, k["features"], rtol=1e-15, atol=0)
        chosen, probs = ias.matnet_predict(k["weights"], ias.density_image(A), ias.density_image(AT), f)
        assert chosen + 1 == k["chosen_algorithm"], (side, probs)


@pytest.mark.parametrize("name", NAMES)
def test_features_and_image_match_oracle(inputs_dir, name):
    A, _ = ias.mtx_read(os.path.join(inputs_dir, name))
    B = transpose(A)
    for X, Y in ((A, B), (B, A)) + (((A, A),) if A.rows == A.cols else ()):
        for n in (26, 18):
            np.testing.assert_array_equal(ias.features(X, Y, n), ob.features(ob.Mat.of(X), ob.Mat.of(Y), n))
    np.testing.assert_array_equal(ias.density_image(A), ob.density_image(ob.Mat.of(A)))
    np.testing.assert_array_equal(ias.density_image(B), ob.density_image(ob.Mat.of(B)))


@pytest.mark.parametrize("case", synthetic(), ids=lambda c: c[0])
def test_features_and_image_synthetic(case):
    _, A = case
    np.testing.assert_array_equal(ias.features(A, A, 26), ob.features(ob.Mat.of(A), ob.Mat.of(A), 26))
    img = ias.density_image(A)
    np.testing.assert_array_equal(img, ob.density_image(ob.Mat.of(A)))
    assert img.sum() == A.nnz or A.rows < 128   # one cell per entry once both sides exceed 128


@pytest.mark.parametrize("weights", sorted(SETS))
def test_matnet_forward_matches_numpy(inputs_dir, weights):
    nf, nc = SETS[weights]
    blob = load_blob(os.path.join(DATA, f"matnet_{weights}.bin"))
    assert blob[:2] == (nf, nc)
    mats = [ias.mtx_read(os.path.join(inputs_dir, n))[0] for n in ("dia.mtx", "LFAT5.mtx", "b1_ss.mtx")]
    mats += [m for _, m in synthetic()]
    for A in mats:
        B = transpose(A)
        f = ias.features(A, B, nf)
        ia, ib = ias.density_image(A), ias.density_image(B)
        chosen, probs = ias.matnet_predict(weights, ia, ib, f)
        ref = np_matnet(blob, ia, ib, f)
        np.testing.assert_allclose(probs, ref, atol=1e-4)
        top2 = np.sort(ref)[-2:]
        if top2[1] - top2[0] > 1e-3:
            assert chosen == int(np.argmax(ref))


def test_blobs_are_the_reference_weights():
    ref = "/root/reference/NetWeights"
    if not os.path.isdir(ref):
        pytest.skip("reference weights not present (GPU box): the blobs were checked where they were made")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import matnet_export as mx
    for name, fn in mx.SETS.items():
        w = mx.arrays(os.path.join(ref, fn))
        _, _, blob = load_blob(os.path.join(DATA, f"matnet_{name}.bin"))
        flat = [a for l in mx.ORDER for a in w[l]]
        assert len(flat) == len(blob)
        for a, b in zip(flat, blob):
            np.testing.assert_array_equal(a.astype(np.float64), b)


def test_matnet_errors(tmp_path):
    net = C.c_void_p()
    assert ias.lib.ias_matnet_load(str(tmp_path / "none.bin").encode(), C.byref(net)) == 5
    bad = tmp_path / "bad.bin"
    bad.write_bytes(b"IASMNET1" + struct.pack("<ii", 26, 5) + b"\0" * 16)
    assert ias.lib.ias_matnet_load(str(bad).encode(), C.byref(net)) == 6
    A = ias.gen_band(16, 1)
    s = A.struct()
    out = np.zeros(26)
    assert ias.lib.ias_features(C.byref(s), C.byref(s), 7, out.ctypes.data_as(ias.f64p)) == 1
