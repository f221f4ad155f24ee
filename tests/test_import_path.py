"""The `globalign` import path: code written against the reference's modules switches
without edits.  Every public name of the reference's src/globalign/{globaligner,conclude,start}.py
(except the per-cell / per-step internals the engine replaces) resolves, to the engine's objects."""
import inspect

import pytest

REFERENCE_NAMES = {
    "globalign.globaligner": ["main", "find_global_alignment", "dp_array_forward", "dp_array_backward",
                              "make_dp_array"],
    "globalign.conclude": ["AlignmentResults", "final_cost_to_score", "final_score_to_cost",
                           "print_nested_list_aligned", "prettify_mat"],
    "globalign.start": ["SimpleScoringSettings", "SimpleCostingSettings", "validate_and_transform_args",
                        "get_common_alphabet", "check_seq_lengths", "read_scoring_mat", "create_scoring_mat",
                        "create_costing_mat", "validate_scoring_mat_keys", "get_max_val", "scoring_mat_to_costing_mat",
                        "costing_mat_to_scoring_mat", "read_seq_from_fasta", "read_first_2_seqs_from_fasta",
                        "draw_random_seq", "draw_two_random_seqs", "make_matrix", "make_3d_array", "check_symmetric",
                        "check_big_main_diag"],
}
# replaced by the device kernels, not exposed: get_next_best_costs (:317-363, one cell),
# cost_ranks_dispatcher (:595-685) and take_* (:688-753) (one traceback step each)


@pytest.mark.parametrize("mod", sorted(REFERENCE_NAMES))
def test_reference_names_resolve(mod):
    import importlib
    m = importlib.import_module(mod)
    for name in REFERENCE_NAMES[mod]:
        assert hasattr(m, name), f"{mod}.{name}"


def test_signatures_match_reference_order():
    from globalign.globaligner import find_global_alignment
    assert list(inspect.signature(find_global_alignment).parameters) == [
        "input_fasta", "output", "seq_1", "seq_2", "scoring_mat_name", "scoring_mat_path", "match_score",
        "mismatch_score", "mismatch_cost", "gap_open_score", "gap_open_cost", "gap_extension_score",
        "gap_extension_cost"]
    from globalign.conclude import AlignmentResults
    assert AlignmentResults._fields == ("seq_1_aligned", "middle_part", "seq_2_aligned", "cost", "score",
                                        "scoring_mat", "costing_mat", "gap_open_score", "gap_open_cost", "output")


def test_global_aligner_devices():
    import globalign
    ga = globalign.GlobalAligner(match_score=2, devices=[0, 0])
    assert ga.devices == [0, 0] and ga.device == 0
    assert globalign.GlobalAligner().devices == [0]
    with pytest.raises(ValueError):
        globalign.GlobalAligner(devices=[])


def test_helpers():
    from globalign.conclude import print_nested_list_aligned
    from globalign.start import make_3d_array, make_matrix
    m = make_matrix(2, 3, 0)
    m[0][0] = 1
    assert m == [[1, 0, 0], [0, 0, 0]]
    a = make_3d_array(2, 2, 3, None)
    a[0][0][0] = 5
    assert a[1][0] == [None] * 3 and a[0][1] == [None] * 3


def test_print_nested_list_aligned(capsys):
    from globalign.conclude import print_nested_list_aligned
    print_nested_list_aligned([[1, 22, "x"], [333, 4, "yy"]])
    assert capsys.readouterr().out == "   1 22  x\n 333  4 yy\n\n"
