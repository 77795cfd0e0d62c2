"""``repic run_ilp`` — drop-in subcommand: the ILP consumer of get_cliques' outputs, with an
exact set-packing solver on the MI355X instead of Gurobi.

Same plugin protocol and arguments as the reference module (repic/commands/run_ilp.py:13-26):
``in_dir``, ``box_size``, ``--num_particles``.  Reads the same four pickles per micrograph
(:29-42,72-80), solves max w.x s.t. A x <= 1, x binary (:50-63) for every micrograph of the
directory in one device batch (repic_amd.ilp), then writes what the reference writes, in its
order: ``<base>.box`` (chosen cliques' consensus coordinates by decreasing confidence, rounded
with np.rint, :112-124) and one more line of ``<base>_runtime.tsv`` (:132-136, the seconds
only, as the reference writes it).  The certification status and gap of each micrograph go to
a sidecar ``<base>_ilp_status.tsv`` (``STATUS\tgap`` per run), which the reference lacks.

Differences, stated: Gurobi stops at a 1e-4 relative MIP gap by default; this solver proves
conflict components of up to 4096 cliques optimal exactly (f32 weights summed in f64) and
picks, among equally good packings, the one its heaviest-first branch order meets first
(Gurobi's choice among ties is unspecified).  Larger components, and components that exceed
``--node_limit``, get a greedy + swap local-search packing (or the branch and bound's best)
certified by a Lagrangian dual bound; the columns that bound leaves within its gap (reduced-
cost fixing) are then searched exactly, which proves most of them optimal.  What remains
within Gurobi's default 1e-4 gap is accepted silently, as Gurobi would; otherwise a warning
names the micrograph and says which case it is.  The search is bounded by node counts only,
so two runs give the same packings.  Lines
of equal confidence follow our clique column order (the reference's is CPython set order,
not reproducible, get_cliques.py:161).  With ``--multi_out`` inputs the
reference raises AttributeError (``confidences`` is a tuple there, :97-106); so does this.
"""
from __future__ import annotations

import glob
import os
import pickle
import sys
import time

import numpy as np

from .. import _lib, ilp
from ..ilp import solve_batch

name = "run_ilp"

# sidecar next to _runtime.tsv: one "STATUS\trelative_gap" line per run_ilp run
STATUS_SUFFIX = "_ilp_status.tsv"
STATUS_NAMES = {ilp.OPTIMAL: "OPTIMAL", ilp.GAP_OK: "GAP_OK", ilp.NODE_LIMIT: "NODE_LIMIT",
                ilp.HEURISTIC: "HEURISTIC"}


def add_arguments(parser):
    """Same CLI surface as the reference (run_ilp.py:16-23) plus tuning knobs."""
    parser.add_argument("in_dir",
                        help="path to input directory containing get_cliques.py output")
    parser.add_argument("box_size", type=int,
                        help="particle detection box size (in int[pixels])")
    parser.add_argument("--num_particles", type=int,
                        help="filter for the number of expected particles (int)")
    parser.add_argument("--node_limit", type=int, default=0,
                        help="branch-and-bound nodes per conflict component (0: the library "
                             "default, 2^14, x4 per reduced-cost-fixing pass); the only limit of the search, so the output does "
                             "not depend on the device's speed or load")
    parser.add_argument("--device", type=int, default=None,
                        help="HIP device (default: $LOCAL_RANK or 0)")


def _load(path):
    with open(path, "rb") as f:
        return pickle.load(f)


def main(args):
    assert os.path.isdir(args.in_dir), "Error - input directory is missing"
    files = glob.glob(os.path.join(args.in_dir, "*_constraint_matrix.pickle"))
    dev = args.device if getattr(args, "device", None) is not None else \
        int(os.environ.get("LOCAL_RANK", "0"))
    # load every micrograph's matrix and weights in the reference's order; a failing load
    # stops there, the earlier micrographs are still solved and written (as the reference
    # would have written them before reaching it)
    t0 = time.time()
    mats, weights, err = [], [], None
    for mf in files:
        try:
            A = _load(mf)
            w = _load(mf.replace("_constraint_matrix", "_weight_vector"))
        except Exception as e:  # noqa: BLE001 - re-raised at this micrograph
            err = e
            break
        mats.append(A)
        weights.append(w)
    xs, status, rgap = [], [], []
    if mats:
        ctx = _lib.Context(dev)
        try:
            xs, status, rgap = solve_batch(ctx, mats, weights, getattr(args, "node_limit", 0),
                                           statuses=True, gaps=True)
        finally:
            ctx.close()
    share = (time.time() - t0) / max(1, len(mats))
    for i, mf in enumerate(files):
        start = time.time()
        base = os.path.basename(mf.replace("_constraint_matrix.pickle", ""))
        print(f"\n--- {base} ---\n")
        if i == len(mats):
            raise err
        A, x = mats[i], xs[i].astype(np.float64)
        if status[i] == ilp.NODE_LIMIT:
            print(f"Warning - {base}: node limit reached in a conflict component and its "
                  f"Lagrangian bound leaves a gap above 1e-4: the packing is the best found, "
                  f"not proven optimal", file=sys.stderr)
        elif status[i] == ilp.HEURISTIC:
            print(f"Warning - {base}: a conflict component of more than "
                  f"{_lib.ilp_big_max()} cliques was not searched; the packing is greedy + "
                  f"swap local search and its Lagrangian bound leaves a gap above 1e-4",
                  file=sys.stderr)
        # run_ilp.py:66-69: every vertex at most once, and at least one clique chosen
        assert np.max(A.tocsr() @ x) == 1, "Error - vertices are assigned to multiple cliques"
        coords = _load(mf.replace("_constraint_matrix", "_consensus_coords"))
        confidences = _load(mf.replace("_constraint_matrix", "_consensus_confidences"))
        multi_out = type(coords[0][0]) == str
        if multi_out:
            coords = coords[1:]
        cliques, confidences = zip(*[(coords[j], confidences[j]) for j in np.where(x == 1.)[0]])
        if multi_out:
            # run_ilp.py:97-106 extends the tuple ``confidences``
            raise AttributeError("'tuple' object has no attribute 'extend'")
        box_size = str(args.box_size)
        out_file = mf.replace("_constraint_matrix.pickle", ".box")
        lines = []
        for j, (val, weight) in enumerate(sorted(zip(cliques, confidences), key=lambda t: t[1],
                                                 reverse=True)):
            if args.num_particles is None or j < args.num_particles:
                lines.append("\t".join([str(int(np.rint(val[0]))), str(int(np.rint(val[1]))),
                                        box_size, box_size, str(weight)]) + "\n")
        with open(out_file, "wt") as o:
            o.writelines(lines)
        # run_ilp.py:132-136 appends the seconds, nothing else; the certification status and
        # the certified relative gap go to a sidecar, so readers of _runtime.tsv are unchanged
        with open(mf.replace("_constraint_matrix.pickle", "_runtime.tsv"), "a") as o:
            o.write(str(share + time.time() - start) + "\n")
        with open(mf.replace("_constraint_matrix.pickle", STATUS_SUFFIX), "a") as o:
            o.write(f"{STATUS_NAMES[status[i]]}\t{rgap[i]:.3e}\n")
    sys.stdout.flush()
