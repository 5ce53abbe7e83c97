"""Deterministic synthetic inputs for Jindo commit parity tests (shared by tests, fixtures
and bench): seeded uniform field elements (Montgomery representatives) and integer noise with
the magnitudes the reference's samplers produce (encoder.go:166-183, prover.go:130-139)."""
import numpy as np


def _uniform_mod(q, n, rng):
    L = (q.bit_length() + 63) // 64
    out = np.zeros((n, L), np.uint64)
    for i in range(n):
        v = int.from_bytes(rng.bytes(8 * L + 8), "little") % q
        for j in range(L):
            out[i, j] = (v >> (64 * j)) & ((1 << 64) - 1)
    return out


def make_v(q, nv, seed):
    return _uniform_mod(q, nv, np.random.default_rng(seed))


def make_randomness(P, q, seed, batch=None, param_sd=False):
    """P: params dict (pyref.JindoParams.as_dict() or fixture).  Returns numpy arrays in the
    layouts of include/ringo.h (leading batch dim if batch is not None).  param_sd: draw with the
    widths the reference's samplers use for these parameters (ecd/ecdBlind for the data columns'
    first/other rows, mask/maskBlind for the mask column, mlwe/maskMLWE; prover.go:93-139)."""
    rng = np.random.default_rng(seed)
    B = 1 if batch is None else batch
    cols, rows, slots, d = P["cols"], P["rows"], P["slots"], P["d"]
    nm = P["in_msis"] + P["mlwe"]
    L = (q.bit_length() + 63) // 64
    last = np.stack([_uniform_mod(q, cols * slots, rng) for _ in range(B)])
    last[:, -1, :] = 0  # genFirstLastRow leaves the last entry zero (prover.go:72)
    mask = np.stack([_uniform_mod(q, rows * slots, rng).reshape(rows, slots, L) for _ in range(B)])
    # encoder Gaussian width ~ b * few (ecdStdDev ~ 2*eta*(b+1)/(b-1)/sqrt(2 pi)); mask columns wider
    if param_sd:
        enc = np.rint(rng.normal(0, P["ecd_sd"], size=(B, cols + 1, rows, d))).astype(np.int64)
        enc[:, :cols, 0] = np.rint(rng.normal(0, P["ecd_blind_sd"], size=(B, cols, d))).astype(np.int64)
        enc[:, cols] = np.rint(rng.normal(0, P["mask_sd"], size=(B, rows, d))).astype(np.int64)
        enc[:, cols, 0] = np.rint(rng.normal(0, P["mask_blind_sd"], size=(B, d))).astype(np.int64)
        mlwe = np.rint(rng.normal(0, P["mlwe_sd"], size=(B, cols + 1, nm, d))).astype(np.int64)
        mlwe[:, cols] = np.rint(rng.normal(0, P["mask_mlwe_sd"], size=(B, nm, d))).astype(np.int64)
    else:
        enc = np.rint(rng.normal(0, 40.0, size=(B, cols + 1, rows, d))).astype(np.int64)
        enc[:, cols] = np.rint(rng.normal(0, 3.0e7, size=(B, rows, d))).astype(np.int64)
        mlwe = np.rint(rng.normal(0, 7.0, size=(B, cols + 1, nm, d))).astype(np.int64)
    out = dict(last_row=last, mask=mask, enc_noise=enc, mlwe_noise=mlwe)
    if batch is None:
        out = {k: v[0] for k, v in out.items()}
    return out
