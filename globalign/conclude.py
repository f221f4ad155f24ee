"""globalign.conclude (reference src/globalign/conclude.py): the result type and score conversions."""
from globalign_amd.results import (AlignmentResults, final_cost_to_score, final_score_to_cost, prettify_mat,
                                   print_nested_list_aligned)

__all__ = ["AlignmentResults", "final_cost_to_score", "final_score_to_cost", "prettify_mat",
           "print_nested_list_aligned"]
