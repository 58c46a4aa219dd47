"""The index / score contract every matcher parity test applies (north_star: bit-exact
correspondence indices).

Correspondence indices (matches0 / matches1, GATs_SuperGlue.py:256-267) must be EQUAL on every
row and column.  A row where neither side reports a match is -1 on both and so equal by
construction; any row that either side matches must match the same index.  The single
exemption is a decision that sits on the threshold itself: the reference's (or the GPU's)
matching score within THR_EPS of match_threshold, where the strict `> 0.2` (:264) is decided
by the last bit of fp32 summation order.  The number of such exempt rows is printed and
returned, so a run shows how often the exemption was used (0 on every committed fixture).

Scores (matching_scores0/1) and conf_matrix: |diff| <= ATOL everywhere (values in [0, 1];
fp32 MFMA products are exact, only the summation order differs from the CPU reference)."""
import numpy as np

ATOL = 2e-5
THR = 0.2
THR_EPS = 1e-6


def assert_indices_exact(got, ref, ref_scores, what, got_scores=None, thr=THR):
    got = np.asarray(got).reshape(-1)
    ref = np.asarray(ref).reshape(-1)
    bad = got != ref
    near = np.abs(np.asarray(ref_scores).reshape(-1) - thr) < THR_EPS
    if got_scores is not None:
        near |= np.abs(np.asarray(got_scores).reshape(-1) - thr) < THR_EPS
    exempt = int((bad & near).sum())
    print(f"{what}: {int(bad.sum())} of {bad.size} differ, {exempt} at the threshold, "
          f"{int((ref > -1).sum())} matched")
    wrong = bad & ~near
    assert not wrong.any(), (f"{what}: {int(wrong.sum())} index mismatches at "
                             f"{np.nonzero(wrong)[0][:10]} (got {got[wrong][:10]}, "
                             f"ref {ref[wrong][:10]})")
    return exempt


def assert_scores_close(got, ref, what, atol=ATOL):
    np.testing.assert_allclose(np.asarray(got), np.asarray(ref), rtol=0, atol=atol, err_msg=what)


def assert_pred_equal(got, ref, what="", thr=THR, atol=ATOL):
    """got / ref: dicts with matches0, matches1, matching_scores0, matching_scores1 of one
    sample (the reference's pred holds batch element 0, GATs_SuperGlue.py:270-273)."""
    n = assert_indices_exact(got["matches0"], ref["matches0"], ref["matching_scores0"],
                             f"{what} matches0", got.get("matching_scores0"), thr)
    n += assert_indices_exact(got["matches1"], ref["matches1"], ref["matching_scores1"],
                              f"{what} matches1", got.get("matching_scores1"), thr)
    assert_scores_close(got["matching_scores0"], ref["matching_scores0"], f"{what} scores0", atol)
    assert_scores_close(got["matching_scores1"], ref["matching_scores1"], f"{what} scores1", atol)
    return n
