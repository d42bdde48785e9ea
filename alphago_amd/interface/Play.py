"""Reference module path ``interface.Play`` (Play.py:5-34).  The reference's
``play_match`` plays one turn of player 1 only (self-declared incorrect, :33);
this one plays whole games (``alphago_amd.search.arena``)."""
from ..search.arena import play_game
from ..search.arena import play_match as play_matches
from ..search.arena import play_match_compat as play_match

__all__ = ["play_match", "play_matches", "play_game"]
