"""Reference module path ``AlphaGo.preprocessing.game_converter`` (game_converter.py:12-214).

``game_converter`` is the reference's (lower-case) class name for the SGF ->
training-HDF5 converter implemented in ``alphago_amd.data.convert`` (own HDF5
writer with LZF, native featurizer); ``run_game_converter`` is its CLI with the
reference flags."""
from ..data.convert import GameConverter, SizeMismatchError, run_game_converter

game_converter = GameConverter

__all__ = ["game_converter", "GameConverter", "SizeMismatchError", "run_game_converter"]

if __name__ == "__main__":
    run_game_converter()
