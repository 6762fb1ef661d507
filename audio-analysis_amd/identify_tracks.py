"""Drop-in for the reference's ``src/identify_tracks.py`` import surface
(``from identify_tracks import classify, get_max_chirps, NON_BIRD,
segment_overlap``, src/analyse.py:10)."""
from aa_amd.identify_tracks import *  # noqa: F401,F403
from aa_amd.identify_tracks import (classify, get_end, get_master_tag, get_max_chirps,  # noqa: F401
                                    load_recording, segment_overlap)
from aa_amd.windows import schedule as load_sample_windows  # noqa: F401
