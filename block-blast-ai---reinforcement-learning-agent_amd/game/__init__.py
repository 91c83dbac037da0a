"""Static game data shared by the host wrappers (the game rules run on the GPU)."""
from .pieces import (  # noqa: F401
    Piece, PIECES, PIECE_LIST, PIECE_NAMES, NUM_PIECES, PIECE_BITS, PIECE_MASKS,
    get_piece_by_name, get_piece_by_index, get_piece_index, get_all_pieces,
    get_random_pieces, piece_to_one_hot, visualize_piece,
)
