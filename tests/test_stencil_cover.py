"""The fused kernel's 2x3 stencil (rgc_fused.hip P1/P2) covers every JI > 0.3 pair (reference
get_cliques.py:40-46): host restatement of its grid plan, f32 keys and half-column test."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_stencil_covers_every_edge():
    import stencil_check
    missed, total = stencil_check.run(seed=7, n_mg=45)
    assert total > 100000 and missed == 0


def test_large_route_stencil_covers_every_edge():
    """Same property for the large-micrograph route's per-picker grids (k1_bin / k2_pairs)."""
    import stencil_check
    missed, total = stencil_check.run(seed=11, n_mg=45, large=True)
    assert total > 100000 and missed == 0
