"""Golden-case definitions shared by ``make_golden.py`` and the parity tests.

A case is a dict: ``box`` (CLI box_size), optional ``flags`` (``--get_cc`` /
``--multi_out``), and an input spec: ``src`` (a committed directory of BOX files),
``synth`` (a :class:`repic_amd.synth.SynthConfig` dict + ``n_mg``), and/or ``files``
(``{relpath: text}`` written verbatim; ``None`` deletes the file).  Inputs are
re-created bit-identically from this spec (checked against ``input_sha256`` in
``meta.json``).

What each case pins (reference file:line in brackets):
* c1_10017*        EMPIAR-10017 example set (config #1) [get_cliques.py:72-229]
* syn_k3           header line [common.py:79-80], Topaz-like negative scores -> numpy
                   sigmoid [common.py:92-94]
* syn_k3_frac      non-integer coordinates, duplicate boxes (degree ties) [:182-183]
* syn_k4/k5/k8     k = 4, 5, 8 cliques [:160-161], even-length medians [:186-190]
* tiny*            graphs with |G| <= 2k nodes: consensus ties broken in graph insertion
                   order instead of set order (networkx FilterAtlas.__iter__)
* ties_getcc       all-identical clusters: every clique ties; largest-CC ties [:151-156]
* skips            missing partner (UnboundLocalError) and empty / blank-first-line
                   files (IndexError) -> empty <base>.box, ids still consumed [:117-130]
* ragged           rows with > 5 tokens are accepted when the shortest row has 5
                   [common.py:81]
* crash_*          reference crash classes and the outputs written before them
"""
from __future__ import annotations

import os
import shutil

HERE = os.path.dirname(os.path.abspath(__file__))


def _syn(**kw):
    base = dict(k=3, n_true=300, box=180, width=4096, height=4096, keep=0.9, jit=0.08,
                fp=0.1, seed=0)
    base.update(kw)
    return base


def _box(lines):
    return "".join(f"{x}\t{y}\t{b}\t{b}\t{s}\n" for x, y, b, s in lines)


CASES = {
    "c1_10017": {"box": 180, "src": "inputs_10017"},
    "c1_10017_getcc": {"box": 180, "src": "inputs_10017", "flags": ["--get_cc"]},
    "c1_10017_multi": {"box": 180, "src": "inputs_10017", "flags": ["--multi_out"]},
    "syn_k3": {"box": 180, "synth": _syn(logit=(2,), header=(1,), seed=11), "n_mg": 4},
    "syn_k3_multi": {"box": 180, "synth": _syn(n_true=120, logit=(1,), seed=12), "n_mg": 3,
                     "flags": ["--multi_out"]},
    "syn_k3_multi_getcc": {"box": 180, "synth": _syn(n_true=120, seed=13), "n_mg": 2,
                           "flags": ["--multi_out", "--get_cc"]},
    "syn_k3_frac": {"box": 150, "synth": _syn(box=150, frac=True, dup=0.1, seed=14), "n_mg": 3},
    "syn_k4": {"box": 176, "synth": _syn(k=4, n_true=450, box=176, width=3838, height=3710,
                                         seed=15), "n_mg": 1},
    "syn_k5": {"box": 180, "synth": _syn(k=5, n_true=200, dup=0.1, seed=16), "n_mg": 2},
    "syn_k8": {"box": 64, "synth": _syn(k=8, n_true=200, box=64, width=1024, height=1024,
                                        keep=0.95, jit=0.06, fp=0.05, dup=0.15, seed=17),
               "n_mg": 1},
    "tiny0": {"box": 100, "synth": _syn(n_true=0, box=100, width=2000, height=2000, keep=1.0,
                                        jit=0.0, fp=0.0, seed=18), "n_mg": 3},
    "tiny1": {"box": 100, "synth": _syn(n_true=1, box=100, width=2000, height=2000, keep=1.0,
                                        jit=0.0, fp=0.0, seed=19), "n_mg": 4},
    "tiny_k4": {"box": 100, "synth": _syn(k=4, n_true=1, box=100, width=2000, height=2000,
                                          keep=1.0, jit=0.0, fp=0.0, seed=20), "n_mg": 4},
    "ties_getcc": {"box": 100, "synth": _syn(n_true=4, box=100, width=2000, height=2000,
                                             keep=1.0, jit=0.0, fp=0.0, seed=21), "n_mg": 6,
                   "flags": ["--get_cc"]},
    "ties": {"box": 100, "synth": _syn(n_true=4, box=100, width=2000, height=2000,
                                       keep=1.0, jit=0.0, fp=0.0, seed=21), "n_mg": 6},
    "skips": {"box": 180, "synth": _syn(n_true=80, width=2048, height=2048, seed=22), "n_mg": 6,
              "files": {"picker1/mg000001.box": None,
                        "picker2/mg000003.box": "",
                        "picker2/mg000004.box": "\n1 2 3 4 5\n"}},
    "ragged": {"box": 100, "files": {
        "a/m1.box": _box([(100, 100, 100, 0.5), (900, 900, 100, 0.4)]).replace(
            "0.5\n", "0.5\textra\ttokens\n"),
        "b/m1.box": _box([(110, 100, 100, 0.6), (905, 900, 100, 0.7)]),
        "c/m1.box": _box([(100, 112, 100, 0.7), (902, 904, 100, 0.2)])}},
    "crash_noedges": {"box": 100, "files": {
        "a/m1.box": _box([(100, 100, 100, 0.5)]), "b/m1.box": _box([(105, 100, 100, 0.6)]),
        "c/m1.box": _box([(100, 103, 100, 0.7)]),
        "a/m2.box": _box([(100, 100, 100, 0.5)]), "b/m2.box": _box([(900, 100, 100, 0.6)]),
        "c/m2.box": _box([(100, 900, 100, 0.7)])}},
    "crash_nocliques": {"box": 100, "files": {
        "a/m1.box": _box([(100, 100, 100, 0.5)]), "b/m1.box": _box([(105, 100, 100, 0.6)]),
        "c/m1.box": _box([(100, 103, 100, 0.7)]),
        "a/m2.box": _box([(100, 100, 100, 0.5)]), "b/m2.box": _box([(105, 100, 100, 0.6)]),
        "c/m2.box": _box([(100, 900, 100, 0.7)])}},
    "crash_ambiguous": {"box": 100, "files": {
        "a/m1.box": _box([(100, 100, 100, 0.5)]), "b/m1.box": _box([(105, 100, 100, 0.6)]),
        "c/m1.box": _box([(100, 103, 100, 0.7)]), "c/m1_copy.box": _box([(1, 1, 100, 0.7)])}},
    "crash_4cols": {"box": 100, "files": {
        "a/m1.box": "100\t100\t100\t0.5\n", "b/m1.box": _box([(105, 100, 100, 0.6)]),
        "c/m1.box": _box([(100, 103, 100, 0.7)])}},
    "crash_blankline": {"box": 100, "files": {
        "a/m1.box": _box([(100, 100, 100, 0.5)]) + "\n" + _box([(300, 300, 100, 0.5)]),
        "b/m1.box": _box([(105, 100, 100, 0.6)]), "c/m1.box": _box([(100, 103, 100, 0.7)])}},
    "crash_headeronly": {"box": 100, "files": {
        "a/m1.box": "x y w h s\n", "b/m1.box": _box([(105, 100, 100, 0.6)]),
        "c/m1.box": _box([(100, 103, 100, 0.7)])}},
}


def materialise(case, in_dir):
    """Create the input directory tree of ``case`` under ``in_dir``."""
    os.makedirs(in_dir, exist_ok=True)
    if "src" in case:
        src = os.path.join(HERE, case["src"])
        for d in sorted(os.listdir(src)):
            if os.path.isdir(os.path.join(src, d)):
                shutil.copytree(os.path.join(src, d), os.path.join(in_dir, d))
    if "synth" in case:
        from repic_amd.synth import SynthConfig, write_box_dirs
        cfg = SynthConfig(**case["synth"])
        write_box_dirs(in_dir, cfg, case["n_mg"])
    for rel, text in case.get("files", {}).items():
        p = os.path.join(in_dir, rel)
        if text is None:
            os.remove(p)
            continue
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(text)
