"""MI355X-native audio-analysis hot path (host side).

Python mirror of the reference's classification surface
(src/identify_tracks.py ``classify``, src/analyse.py CLI) over libaa.so, the
HIP/gfx950 front end + CNN behind a C ABI (include/aa.h).
"""
__version__ = "0.1.0"
