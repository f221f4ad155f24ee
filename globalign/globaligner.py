"""globalign.globaligner (reference src/globalign/globaligner.py): the API and the CLI entry point.

find_global_alignment (:132-314), make_dp_array (:756-821), dp_array_forward (:366-392),
dp_array_backward (:395-593) and main (:23-129, the `globaligner` console script) from
globalign_amd.globaligner."""
import sys

from globalign_amd.globaligner import (GlobalAligner, dp_array_backward, dp_array_forward, find_global_alignment,
                                       main, make_dp_array)
from globalign_amd.results import AlignmentResults, final_cost_to_score
from globalign_amd.scoring import get_max_val, make_matrix, validate_and_transform_args

__all__ = ["find_global_alignment", "make_dp_array", "dp_array_forward", "dp_array_backward", "main",
           "GlobalAligner", "AlignmentResults", "final_cost_to_score", "get_max_val", "make_matrix",
           "validate_and_transform_args"]

if __name__ == "__main__":
    sys.exit(main())
