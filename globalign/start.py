"""globalign.start (reference src/globalign/start.py): validation, matrices, FASTA, synthetic inputs."""
from globalign_amd.random_seqs import draw_random_seq, draw_two_random_seqs
from globalign_amd.scoring import (SimpleCostingSettings, SimpleScoringSettings, check_big_main_diag,
                                   check_seq_lengths, check_symmetric, costing_mat_to_scoring_mat, create_costing_mat,
                                   create_scoring_mat, get_common_alphabet, get_max_val, make_3d_array, make_matrix,
                                   read_first_2_seqs_from_fasta, read_scoring_mat, read_seq_from_fasta,
                                   scoring_mat_to_costing_mat, validate_and_transform_args, validate_scoring_mat_keys)

__all__ = ["SimpleScoringSettings", "SimpleCostingSettings", "validate_and_transform_args", "get_common_alphabet",
           "check_seq_lengths", "read_scoring_mat", "create_scoring_mat", "create_costing_mat",
           "validate_scoring_mat_keys", "get_max_val", "scoring_mat_to_costing_mat", "costing_mat_to_scoring_mat",
           "read_seq_from_fasta", "read_first_2_seqs_from_fasta", "draw_random_seq", "draw_two_random_seqs",
           "make_matrix", "make_3d_array", "check_symmetric", "check_big_main_diag"]
