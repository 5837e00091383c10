"""CPU: the native read.big.matrix(sep='\\t') reader (tp_tsv_dims / tp_read_tsv,
R/TADpole.R:17,160).  Host code only: runs without a GPU.  Expected values are
Python's float() of each field (correctly rounded, as std::from_chars) with R's
NA rules: NA / NaN / empty / non-numeric -> NaN, Inf spellings -> +-inf."""
import ctypes

import numpy as np
import pytest

from tadpole_amd import _lib, api
from tadpole_amd._lib import cint, dp


def _expected(text):
    rows = [ln for ln in text.replace("\r\n", "\n").rstrip("\n").split("\n")]
    ncol = len(rows[0].split("\t"))
    out = np.full((len(rows), ncol), np.nan)
    for i, ln in enumerate(rows):
        for j, f in enumerate(ln.split("\t")):
            f = f.strip().strip('"')
            try:
                v = float(f)
                if f.lower() in ("nan", "+nan", "-nan"):
                    v = np.nan
            except ValueError:
                v = np.nan
            out[i, j] = v
    return out


CASES = {
    "ints": "1\t2\t3\n4\t5\t6\n",
    "decimals_exp": "0.1\t-2.5e-3\t1E5\n3.14159265358979\t+7\t-0\n",
    "na_forms": "NA\tNaN\t\nnan\t12\tfoo\n",
    "inf": "Inf\t-Inf\t1\n2\tInfinity\t-Infinity\n",
    "crlf_no_final_newline": "1\t2\r\n3\t4",
    "short_line": "1\t2\t3\n4\n",
    "big_ints": "123456789012345\t9007199254740993\t-42\n",
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_read_tsv_cases(tmp_path, name):
    text = CASES[name]
    p = tmp_path / f"{name}.tsv"
    p.write_bytes(text.encode())
    got = api.read_matrix(p)
    exp = _expected(text)
    assert got.shape == exp.shape
    assert np.array_equal(got, exp, equal_nan=True), (got, exp)


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_read_tsv_random_matches_numpy(tmp_path, threads):
    rng = np.random.default_rng(threads)
    m = rng.poisson(3.0, (700, 700)).astype(float)
    m[rng.random(m.shape) < 0.01] = np.nan
    m[:, 5] = rng.standard_normal(700) * 1e-7           # decimals with exponents
    p = tmp_path / "m.tsv"
    np.savetxt(p, m, delimiter="\t", fmt="%.17g")
    got = api.read_matrix(p, nthreads=threads)
    assert np.array_equal(got, m, equal_nan=True)


def test_read_tsv_column_major_layout(tmp_path):
    m = np.arange(12.0).reshape(3, 4)
    p = tmp_path / "c.tsv"
    np.savetxt(p, m, delimiter="\t", fmt="%g")
    L = _lib.load()
    path = ctypes.c_char_p(str(p).encode())
    out = np.zeros(12)
    st = cint(0)
    L.tp_read_tsv(ctypes.byref(path), ctypes.byref(cint(3)), ctypes.byref(cint(4)), ctypes.byref(cint(2)),
                  ctypes.byref(cint(0)), dp(out), ctypes.byref(st))
    _lib.check(st)
    assert np.array_equal(out.reshape(4, 3).T, m)      # R's column-major matrix


def test_read_tsv_errors(tmp_path):
    p = tmp_path / "long.tsv"
    p.write_bytes(b"1\t2\n3\t4\t5\n")
    with pytest.raises(_lib.TadpoleError):
        api.read_matrix(p)
    with pytest.raises(_lib.TadpoleError):
        api.read_matrix(tmp_path / "missing.tsv")


def test_read_tsv_empty(tmp_path):
    p = tmp_path / "e.tsv"
    p.write_bytes(b"")
    assert api.read_matrix(p).shape == (0, 0)
