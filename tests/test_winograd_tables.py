"""The Winograd F(m, 3) tables the split-bf16 kernels compile in
(audio-analysis_amd/csrc/aa_conv_wg.h: wg_bt = B^T, wg_at = A^T, wg_g = G)
reproduce the kernel-width-3 correlation y_k = sum_t g_t d_{k+t} exactly
(rational arithmetic on the parsed tables), and the factored F(6, 3) input
transform conv_wg / conv_wgf stage with equals B^T d.  CPU only: the tables
are read from the header text."""
import re
from fractions import Fraction
from pathlib import Path

import numpy as np
import pytest

HDR = Path(__file__).resolve().parents[1] / "audio-analysis_amd" / "csrc" / "aa_conv_wg.h"


def _num(tok):
    tok = tok.strip().rstrip("f")
    if "/" in tok:
        a, b = tok.split("/")
        return Fraction(a.strip()) / Fraction(b.strip())
    return Fraction(tok)


def _table(name, rows, cols):
    src = HDR.read_text()
    m = re.search(rf"{name}\[{rows}\]\[{cols}\]\s*=\s*\{{(.*?)\}};", src, re.S)
    assert m, name
    body = m.group(1).replace("{", " ").replace("}", " ")
    vals = [_num(t) for t in body.split(",") if t.strip()]
    assert len(vals) == rows * cols, (name, len(vals))
    return [vals[r * cols:(r + 1) * cols] for r in range(rows)]


FORMS = {2: ("b2", "a2", "g2"), 3: ("b3", "a3", "g3"), 4: ("b4", "a4", "g4"), 6: ("b6", "a6", "g6")}


@pytest.mark.parametrize("m", [2, 3, 4, 6])
def test_tables_compute_the_correlation(m):
    a = m + 2
    bn, an, gn = FORMS[m]
    BT, AT, G = _table(bn, a, a), _table(an, m, a), _table(gn, a, 3)
    rng = np.random.default_rng(m)
    for _ in range(5):
        d = [Fraction(int(v)) for v in rng.integers(-50, 50, a)]
        g = [Fraction(int(v)) for v in rng.integers(-50, 50, 3)]
        u = [sum(BT[e][t] * d[t] for t in range(a)) for e in range(a)]
        v = [sum(G[e][k] * g[k] for k in range(3)) for e in range(a)]
        y = [sum(AT[k][e] * u[e] * v[e] for e in range(a)) for k in range(m)]
        assert y == [sum(g[t] * d[k + t] for t in range(3)) for k in range(m)]


def test_factored_f63_input_transform():
    """conv_wg's staging (and conv_wgf's transform MFMA operand) use the F(6, 3)
    input transform in factored form: the same u = B^T d."""
    BT = _table("b6", 8, 8)
    rng = np.random.default_rng(7)
    for _ in range(20):
        d = [Fraction(int(v), 4) for v in rng.integers(-400, 400, 8)]
        d0, d1, d2, d3, d4, d5, d6, d7 = d
        a12, b12 = d2 + d6 - Fraction(17, 4) * d4, d1 + d5 - Fraction(17, 4) * d3
        a34 = d6 + Fraction(1, 4) * d2 - Fraction(5, 4) * d4
        b34 = Fraction(1, 2) * d1 - Fraction(5, 2) * d3 + 2 * d5
        a56 = d6 + 4 * d2 - 5 * d4
        b56 = 2 * d1 - Fraction(5, 2) * d3 + Fraction(1, 2) * d5
        u = [d6 - d0 + Fraction(21, 4) * (d2 - d4), a12 + b12, a12 - b12, a34 + b34, a34 - b34, a56 + b56,
             a56 - b56, d7 - d1 + Fraction(21, 4) * (d3 - d5)]
        assert u == [sum(BT[e][t] * d[t] for t in range(8)) for e in range(8)]


def test_bt_entries_exact_in_bf16():
    """conv_wgf feeds B^T to a bf16 MFMA as its B operand: every entry must be
    a bf16 number (8 significant bits)."""
    for m, (bn, _, _) in FORMS.items():
        for row in _table(bn, m + 2, m + 2):
            for x in row:
                f = np.float32(float(x))
                assert float(x) == float(f)
                bits = f.view(np.uint32)
                assert bits & 0xFFFF == 0, (m, x)
