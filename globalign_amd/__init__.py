"""globalign_amd -- MI355X-native engine behind globalign's alignment API.

    from globalign_amd import find_global_alignment, GlobalAligner
"""
from .globaligner import (GlobalAligner, __version__, dp_array_backward, dp_array_forward, find_global_alignment,
                          make_dp_array)
from .random_seqs import draw_random_seq, draw_two_random_seqs
from .results import AlignmentResults, final_cost_to_score, final_score_to_cost

__all__ = ["GlobalAligner", "find_global_alignment", "AlignmentResults", "make_dp_array", "dp_array_forward",
           "dp_array_backward", "final_cost_to_score", "final_score_to_cost", "draw_random_seq", "draw_two_random_seqs",
           "__version__"]
