"""CPU-only checks of the drop-in boundary: the C-ABI library loads and exports every entry
point include/gi.h declares, and the flag parser matches the reference's ParseArgs
(utils/io_utils.cpp:16-212) as restated by the oracle."""
import ctypes as C
import os
import re

import pytest

import gi_amd
import oracle_lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "gi.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gi_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    L = gi_amd.lib()
    syms = declared_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(gi_amd.EXPORTED) == syms


def test_photon_record_layout():
    assert gi_amd.PHOTON_DTYPE.itemsize == 20
    assert C.sizeof(gi_amd.GiParams) == 34 * 4 + 9 * 8 + 8


ARGSETS = [
    ["a.scn", "b.png"],
    ["a.scn", "b.png", "-v", "-threads", "8", "-aa", "-3", "-real", "-no_fresnel", "-ir", "1.2"],
    ["a.scn", "b.png", "-no_ambient", "-no_direct", "-no_transmissive", "-no_specular",
     "-no_indirect", "-no_caustic", "-photon_viz", "-cache", "-no_monte"],
    ["a.scn", "b.png", "-fast_global", "-md", "0", "-absorb", "-1", "-no_rs", "-no_dt", "-tt",
     "0", "-no_ds", "-st", "7"],
    ["a.scn", "b.png", "-global", "1000000", "-caustic", "0", "-pd", "5", "-it", "32", "-gs",
     "64", "-gd", "-1", "-gf", "cone", "0.5", "-cs", "100", "-cd", "0.3", "-cf", "gauss"],
    ["a.scn", "b.png", "-no_shadow", "-no_ss", "-lt", "0", "-ss", "-4", "-dof", "4", "12.5",
     "0.05", "-resolution", "-640", "480", "-seed", "42"],
    ["a.scn", "b.png", "-gf", "gauss", "-cf", "cone", "2.5", "-dof", "0", "0", "0"],
]


@pytest.mark.parametrize("args", ARGSETS)
def test_parse_args_matches_reference_restatement(args):
    p, sc, out, w, h, aa, real = gi_amd.ParseArgs(args)
    rc, q, w2, h2, aa2, real2 = oracle_lib.parse_args(args)
    assert rc == 0
    assert (sc, out) == ("a.scn", "b.png")
    assert (w, h, aa, real) == (w2, h2, aa2, real2)
    for f, _ in gi_amd.GiParams._fields_:
        assert getattr(p, f) == getattr(q, f), f


@pytest.mark.parametrize("args", [["a.scn", "b.png", "-bogus"], ["a.scn", "b.png", "c.png"]])
def test_parse_args_rejects_like_reference(args):
    with pytest.raises(ValueError, match="Invalid program argument"):
        gi_amd.ParseArgs(args)
    assert oracle_lib.parse_args(args)[0] == 1


def test_parse_args_usage():
    with pytest.raises(ValueError, match="Usage"):
        gi_amd.ParseArgs(["only.scn"])


def test_write_image_png_roundtrip(tmp_path):
    import numpy as np
    from pngio import read_png
    rgb = (np.arange(5 * 7 * 3) % 251).astype(np.uint8).reshape(5, 7, 3)
    p = str(tmp_path / "x.png")
    gi_amd.write_image(p, rgb)
    back = read_png(p)
    np.testing.assert_array_equal(back, rgb[::-1])  # bottom-up rows, R2Image.cpp:1430
