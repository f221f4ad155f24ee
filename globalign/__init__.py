"""Drop-in import path for code written against globalign (iamgiddyaboutgit/globalign).

    from globalign.globaligner import find_global_alignment     # globaligner.py:132-314
    from globalign.conclude import AlignmentResults             # conclude.py:7-151
    from globalign.start import validate_and_transform_args     # start.py:150-353
    import globalign; globalign.GlobalAligner(devices=[0, 1])   # north_star's name

Every name resolves to the MI355X engine in globalign_amd; the DP fill and traceback run on the GPU
(no CPU fallback).  Install only one of globalign / globalign_amd on a path: this package shadows
the pure-Python reference of the same name.
"""
from globalign_amd import (AlignmentResults, GlobalAligner, __version__, dp_array_backward, dp_array_forward,
                           find_global_alignment, make_dp_array)

__all__ = ["AlignmentResults", "GlobalAligner", "find_global_alignment", "make_dp_array", "dp_array_forward",
           "dp_array_backward", "__version__"]
