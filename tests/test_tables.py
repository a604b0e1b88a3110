"""CPU: the generated VP8 constant tables (webp_amd/csrc/vp8_tables.h, oracle/
vp8_tables.h) are identical to each other and, where the reference checkout
is present, to the values its Go source declares (tools/gen_vp8_tables.py)."""
import os
import sys

import pytest

from conftest import REFERENCE, ROOT


def test_product_and_oracle_tables_identical():
    a = open(os.path.join(ROOT, "webp_amd", "csrc", "vp8_tables.h")).read()
    b = open(os.path.join(ROOT, "oracle", "vp8_tables.h")).read()
    assert a == b and "vp8_coeffs_proba0[1056]" in a


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference checkout not present")
def test_tables_match_reference_source():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_vp8_tables as G
    srcs = {f: G.strip_comments(open(os.path.join(G.REF, f)).read()) for f in ("constants.go", "proba.go")}
    syms = G.symbols(srcs["constants.go"])
    tabs = [(c, t, G.values(srcs[f], g, syms)) for f, g, c, t in G.TABLES]
    for f, g, c, t in G.ENC_TABLES:
        src = G.strip_comments(open(os.path.join(os.path.dirname(G.REF), f)).read())
        tabs.append((c, t, G.values(src, g, syms)))
    txt = open(os.path.join(ROOT, "webp_amd", "csrc", "vp8_tables.h")).read()
    for cname, ctype, vals in tabs:
        start = txt.index(f"{cname}[")
        body = txt[txt.index("{", start) + 1:txt.index("};", start)]
        assert [int(x) for x in body.replace(",", " ").split()] == vals, cname
