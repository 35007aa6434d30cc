"""Collation weights pinned independently of the generated tables (CPU).

tests/golden/collation_pin.json holds per-plane digests of every BMP code point's one-character
sort key under utf8mb4_general_ci, utf8mb4_unicode_ci and utf8mb4_0900_ai_ci, made by
tests/golden/make_collation_pin.py from the reference's CollationLUT.cpp compiled as it lies
(not from tools/gen_collation_data.py's run encoding, which both the device headers and the oracle
compile).  Checked here:

* the oracle's orc_collate for all 3 x 65536 code points;
* both copies of the generated headers (tiflash_amd/csrc/ — what the device compiles — and
  oracle/), expanded from their runs;
* that the check is sensitive: a single corrupted run fails it."""
import ctypes
import json
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import make_collation_pin as mcp  # noqa: E402  (key rules only; nothing from /root/reference)

PIN = json.load(open(os.path.join(ROOT, "tests", "golden", "collation_pin.json")))
COLLATORS = {"general_ci": 3, "unicode_ci": 4, "uca0900_ai_ci": 5}  # tfg_collator


def _utf8(cp):
    return chr(cp).encode("utf-8", "surrogatepass")


@pytest.mark.parametrize("name", list(COLLATORS))
def test_oracle_collate_matches_pin(orc, name):
    f = orc.lib().orc_collate
    f.restype = ctypes.c_size_t
    f.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p]
    out = ctypes.create_string_buffer(64)
    keys = {}

    def key(cp):
        s = _utf8(cp)
        n = f(COLLATORS[name], s, len(s), len(s), out)
        return out.raw[:n]

    got = mcp.plane_digests(key)
    bad = [p for p in range(256) if got[p] != PIN[name][p]]
    assert not bad, f"{name}: planes {[hex(p) for p in bad[:8]]} differ from the pin"
    del keys


def _gci_runs(path):
    text = open(path).read()
    body = text[text.index("#define TFG_GCI_RUNS_INIT"):]
    return [tuple(int(x) for x in m) for m in re.findall(r"\{(\d+), (\d+), (\d+)\}", body)]


def _gci_lut(runs):
    lut = list(range(65536))
    for a, b, kv in runs:
        kind, val = kv >> 16, kv & 0xFFFF
        for x in range(a, b + 1):
            lut[x] = val if kind else (x + (val - 65536 if val >= 32768 else val)) & 0xFFFF
    return lut


def _uca(path, tag):
    text = open(path).read()
    size = int(re.search(r"#define TFG_UCA%s_SIZE (\d+)" % tag, text).group(1))
    rb = text.index("#define TFG_UCA%s_RUNS_INIT" % tag)
    re_ = text.index("#define TFG_UCA%s_NLONG" % tag)
    runs = [(int(a), int(n), int(b, 16), int(d, 16))
            for a, n, b, d in re.findall(r"\{(\d+), (\d+), 0x([0-9a-f]+)ull, 0x([0-9a-f]+)ull\}", text[rb:re_])]
    lb = text.index("#define TFG_UCA%s_LONG_INIT" % tag)
    le = text.find("#define", lb + 10)
    longs = {int(c, 16): (int(x, 16), int(y, 16))
             for c, x, y in re.findall(r"\{0x([0-9a-f]+), 0x([0-9a-f]+)ull, 0x([0-9a-f]+)ull\}",
                                       text[lb:le if le > 0 else len(text)])}
    return size, runs, longs


def _uca_lut(size, runs):
    lut = [0] * size
    for st, n, base, d in runs:
        for k in range(n):
            lut[st + k] = (base + k * d) % (1 << 64)
    return lut


def _header_digests(csrc_dir, corrupt=None):
    gr = _gci_runs(os.path.join(csrc_dir, "collation_data.h"))
    if corrupt == "gci":  # one run's value off by one
        i = next(j for j, r in enumerate(gr) if r[0] <= 0xE0 <= r[1])  # the run holding 'à' 
        a, b, kv = gr[i]
        gr[i] = (a, b, kv ^ 1)
    g = _gci_lut(gr)
    out = {"general_ci": mcp.plane_digests(lambda cp: mcp.key_general_ci(g, cp))}
    for tag, name, pad in (("0400", "unicode_ci", True), ("0900", "uca0900_ai_ci", False)):
        size, runs, longs = _uca(os.path.join(csrc_dir, "uca_data.h"), tag)
        if corrupt == tag:  # a run inside the CJK compatibility block, base off by one
            i = next(j for j, r in enumerate(runs) if r[0] <= 0x4E10 < r[0] + r[1])
            st, n, base, d = runs[i]
            runs[i] = (st, n, base + 1, d)
        lut = _uca_lut(size, runs)
        out[name] = mcp.plane_digests(lambda cp: mcp.key_uca(lut, longs, cp, pad))
    return out


@pytest.mark.parametrize("where", ["tiflash_amd/csrc", "oracle"])
def test_generated_headers_match_pin(where):
    got = _header_digests(os.path.join(ROOT, where))
    for name in COLLATORS:
        bad = [p for p in range(256) if got[name][p] != PIN[name][p]]
        assert not bad, f"{where} {name}: planes {[hex(p) for p in bad[:8]]} differ from the pin"


@pytest.mark.parametrize("corrupt,name,plane", [("gci", "general_ci", 0x00), ("0400", "unicode_ci", 0x4E),
                                                ("0900", "uca0900_ai_ci", 0x4E)])
def test_corrupted_run_fails_the_pin(corrupt, name, plane):
    got = _header_digests(os.path.join(ROOT, "tiflash_amd", "csrc"), corrupt=corrupt)
    bad = [p for p in range(256) if got[name][p] != PIN[name][p]]
    assert plane in bad, (corrupt, [hex(p) for p in bad])  # (a run may span several planes)


def test_pin_long_weights_match_headers():
    for tag in ("0400", "0900"):
        for where in ("tiflash_amd/csrc", "oracle"):
            _, _, longs = _uca(os.path.join(ROOT, where, "uca_data.h"), tag)
            want = {int(k, 16): (int(a, 16), int(b, 16)) for k, (a, b) in PIN["long_" + tag].items()}
            assert longs == want, (where, tag)
