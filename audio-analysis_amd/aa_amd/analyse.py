"""``analyse.py`` CLI and result post-processing on the MI355X path.

Surface kept from the reference (src/analyse.py):
  analyse.py FILE [--bird-model PATH]* [-o] [--analyse-tracks BOOL]
             [--old-cacophony-index]                               :382-420
  examine / species_identify / filter_by_location / species_by_location /
  find_square / merge_neighbours / calc_cacophony_index / filter_tracks /
  get_chirps                                                        :18-373
The JSON written (FILE.txt["analysis_result"], or stdout with -o) has the
reference's keys and version strings.  Everything here is host bookkeeping
over classify()'s results; the compute is in classify() (GPU).
"""
from __future__ import annotations

import argparse
import json
import logging
import math
import os
import sys
import time
from pathlib import Path

from .identify_tracks import NON_BIRD, classify, get_max_chirps, segment_overlap

SPECIES_IDENTIFY_VERSION = "2025-12-01"


def calc_cacophony_index(tracks, length):
    """Percent of each 20 s period covered by (bird) tracks (src/analyse.py:18-77)."""
    version = "1.0"
    period = 20
    bins = math.ceil(length / period)
    last_bin = None
    if bins > 1 and length - period * (bins - 1) < 2:  # fold a short tail into the last bin
        bins -= 1
        last_bin = length
    percents = [{"begin_s": i * period, "end_s": min(length, (i + 1) * period), "index_percent": 0}
                for i in range(bins)]
    if last_bin is not None:
        percents[-1]["end_s"] = last_bin
    idx = 0
    span_len = period
    if percents:
        span_len = percents[idx]["end_s"] - percents[idx]["begin_s"]
    idx_end = span_len
    covered = 0
    until = -1
    for track in tracks:
        if until >= track.start and until < track.end:
            seg = (until, track.end)
        elif until < track.end:
            seg = (track.start, track.end)
        else:
            continue
        while seg[1] > idx_end:
            if seg[0] < idx_end:
                covered += idx_end - seg[0]
                seg = (idx_end, seg[1])
            percents[idx]["index_percent"] = round(100 * covered / span_len, 1)
            covered = 0
            idx = min(idx + 1, bins - 1)
            span_len = percents[idx]["end_s"] - percents[idx]["begin_s"]
            idx_end += span_len
        covered += seg[1] - seg[0]
        until = seg[1]
        idx = min(len(percents) - 1, int(until / span_len))
        idx = min(idx, bins - 1)
        span_len = percents[idx]["end_s"] - percents[idx]["begin_s"]
    if idx < len(percents):
        percents[idx]["index_percent"] = round(100 * covered / span_len, 1)
    return percents, version


def filter_tracks(tracks):
    return [t for t in tracks if t.master_tag is not None and t.master_tag.what not in NON_BIRD]


def get_chirps(tracks, bird_labels, signals):
    """Signals overlapping bird-tagged tracks, each counted once (:80-117)."""
    birds = sorted((t for t in tracks if t.master_tag is not None and t.master_tag.what in bird_labels),
                   key=lambda t: t.start)
    last_end = 0
    chirps = 0
    for t in birds:
        start, end = t.start, t.end
        if start < last_end:
            start = last_end
            end = max(start, end)
        i = 0
        while i < len(signals):
            s = signals[i]
            if segment_overlap((start, end), (s.start, s.end)) > 0 and t.mel_freq_overlap(s) > -200:
                chirps += 1
                del signals[i]
            elif s.start > end:
                break
            else:
                i += 1
        last_end = t.end
    return chirps


def _species_file():
    env = os.environ.get("AA_EBIRD_SPECIES")
    return Path(env) if env else Path("./src/ebird_species.json")


def find_square(squares, lng, lat):
    """Binary search of lng-sorted atlas squares, then a local scan on lat (:241-278)."""
    high, low, found = len(squares), 0, None
    while high >= low:
        mid = (high + low) // 2
        b = squares[mid]["bounds"]
        if b[0] <= lng and b[2] >= lng:
            found = mid
            break
        if b[2] < lng:
            low = mid + 1
        else:
            high = mid - 1
    if found is None:
        logging.error("Could not find species square for %s, %s", lng, lat)
        return None
    decrement = False
    while True:
        if mid < 0:
            return None
        if mid < len(squares):
            b = squares[mid]["bounds"]
        if mid > len(squares) or b[0] > lng:
            if decrement:
                return None
            decrement = True
            mid = found - 1
            continue
        if b[1] <= lat and b[3] >= lat:
            return squares[mid]
        mid = mid - 1 if decrement else mid + 1


def merge_neighbours(square, species_meta):
    per_month = square["species_per_month"]
    for nb in square["neighbours_i"]:
        for species, months in species_meta[nb]["species_per_month"].items():
            if species not in per_month:
                per_month[species] = months.copy()
                continue
            for m, c in months.items():
                per_month[species][m] += c
    return per_month


def species_by_location(rec_metadata):
    species_file = _species_file()
    if not species_file.exists():
        logging.info("No species file")
        return None, None
    with species_file.open("r") as f:
        species_data = json.load(f)
    loc = rec_metadata.get("location")
    species_list = set()
    region_code = None
    if loc is None:
        region_code = "NZ"
        logging.info("No location data assume nz species")
        for info in species_data.values():
            r = info["region"]["info"]
            parent = r.get("parent")
            if (r["type"] == "country" and r["code"] == region_code) or (
                    parent is not None and parent["code"] == region_code):
                species_list.update(info["species"])
        return list(species_list), region_code
    lat, lng = loc.get("lat"), loc.get("lng")
    square_file = species_file.parent / "ebird_species_per_square.json"
    if square_file.exists():
        with square_file.open("r") as f:
            squares = json.load(f)
        sq = find_square(squares, lng, lat)
        if sq is not None:
            per_month = merge_neighbours(sq, squares)
            total = sum(sum(m.values()) for m in per_month.values())
            if total < 30 and len(per_month) > 3:
                logging.info("Not using atlas square filtering as data is incomplete, falling back to region")
            else:
                logging.info("Found species list of %s", list(per_month.keys()))
                return list(per_month.keys()), sq["region_code"]
    for code, info in species_data.items():
        b = info["region"]["info"]["bounds"]
        if b["minX"] <= lng <= b["maxX"] and b["minY"] <= lat <= b["maxY"]:
            species_list = info["species"]
            region_code = code
            logging.info("Match lat %s lng %s to region %s ", lat, lng, info)
            break
    return species_list, region_code


def filter_by_location(meta_data, tracks):
    """Mark predictions whose eBird species is not seen in the recording's
    region as filtered; add a generic "bird" when every specific one is
    filtered (:178-238)."""
    observed, region_code = species_by_location(meta_data)
    if region_code is None:
        return
    for track in tracks:
        for mr in track.results:
            if len(mr.predictions) == 0:
                continue
            any_filtered = False
            for p in mr.predictions:
                if p.ebird_id is None or any(e in observed for e in p.ebird_id):
                    continue
                any_filtered = True
                p.filtered = True
                logging.info("Region filtering %s ebird %s", p.what, p.ebird_id)
            if any_filtered and not any(p.what == "bird" for p in mr.predictions):
                logging.info("Adding bird as specific bird labels were filtered")
                conf = max(p.confidence for p in mr.predictions if p.filtered)
                thr = max(p.threshold_used for p in mr.predictions if p.threshold_used)
                mr.add_prediction("bird", conf, None, thr, normalize_confidence=False)


def read_sidecar(file_name):
    """The recording's FILE.txt metadata (tracks, location), or None (:132-137)."""
    meta_file = Path(file_name).with_suffix(".txt")
    if meta_file.exists():
        with meta_file.open("r") as f:
            return json.load(f)
    return None


def species_identify(file_name, bird_models, analyse_tracks):
    meta_data = read_sidecar(file_name)
    res = classify(file_name, bird_models, analyse_tracks, meta_data) if bird_models is not None else None
    return species_result(res, meta_data, analyse_tracks, bird_models is not None)


def _signal_arrays(signals):
    """[s.to_array() for s in signals] (rounded to 0.1 as the reference's
    Signal.to_array, :944-951) in one numpy rounding: the same np.float64
    elements when every row is a float row (a float start makes it one);
    otherwise row by row."""
    if not signals or any(type(s.start) is not float for s in signals):
        return [s.to_array() for s in signals]
    import numpy as np
    return [list(r) for r in np.round(np.array([[s.start, s.end, s.freq_start, s.freq_end] for s in signals]), 1)]


def species_result(res, meta_data, analyse_tracks, have_models=True):
    """species_identify's result document from classify()'s return value
    (src/analyse.py:129-175); shared by the per-file path and the batched
    corpus runner (aa_amd.batch), so both write the same JSON."""
    labels = []
    result = {}
    region_code = None
    if have_models:
        if res is not None:
            tracks, length, signals, raw_length, bird_labels = res
            if meta_data is not None:
                filter_by_location(meta_data, tracks)
            for t in tracks:
                t.set_master_tag()
            rec_signals = _signal_arrays(signals)
            chirps = get_chirps(tracks, bird_labels, signals)
            cacophony_index, version = calc_cacophony_index(filter_tracks(tracks), length)
            labels.extend(t.get_meta() for t in tracks)
            if not analyse_tracks:
                max_chirps = get_max_chirps(length)
                if region_code is not None:
                    result["region_code"] = region_code
                result["duration"] = raw_length
                result["cacophony_index"] = cacophony_index
                result["cacophony_index_version"] = "2.0"
                result["chirps"] = {"chirps": chirps, "max_chirps": max_chirps,
                                    "chirp_index": 0 if max_chirps == 0 else round(100 * chirps / max_chirps),
                                    "signals": rec_signals}
    result["non_bird_tags"] = NON_BIRD
    result["species_identify"] = labels
    result["species_identify_version"] = SPECIES_IDENTIFY_VERSION
    return result


def examine(file_name, bird_model, analyse_tracks=False):
    summary = {}
    summary.update(species_identify(file_name, bird_model, analyse_tracks))
    return summary


def none_or_str(value):
    return None if value.lower() in ("none", "null") else value


def str2bool(v):
    if isinstance(v, bool):
        return v
    if v.lower() in ("yes", "true", "t", "y", "1"):
        return True
    if v.lower() in ("no", "false", "f", "n", "0"):
        return False
    raise argparse.ArgumentTypeError("Boolean value expected.")


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-o", "--meta-to-stdout", action="count",
                    help="Print metadata to stdout instead of saving to file.")
    ap.add_argument("--old-cacophony-index", action="count",
                    help="Calculate old cacophony index on this file")
    ap.add_argument("--bird-model", type=none_or_str, action="append", help="Path to bird model")
    ap.add_argument("file", help="Audio file to run on")
    ap.add_argument("--analyse-tracks", type=str2bool, default=False,
                    help="Classify human made tracks marked with classify flag, in metadata file")
    args = ap.parse_args(argv)
    if args.bird_model is None or len(args.bird_model) == 0:
        args.bird_model = ["/models/pre-model/audioModel.keras", "/models/bird-model-v2m/audioModel.keras"]
    return args


def init_logging():
    logging.basicConfig(stream=sys.stderr, level=logging.INFO,
                        format="%(process)d %(thread)s:%(levelname)7s %(message)s",
                        datefmt="%Y-%m-%d %H:%M:%S")


def main(argv=None):
    args = parse_args(argv)
    init_logging()
    t0 = time.time()
    if args.old_cacophony_index:
        raise NotImplementedError("--old-cacophony-index (ffmpeg/opusdec DCT index) is out of scope")
    summary = examine(args.file, args.bird_model, analyse_tracks=args.analyse_tracks)
    summary["processing_time_seconds"] = round(time.time() - t0, 1)
    if args.meta_to_stdout:
        print(json.dumps(summary, sort_keys=True, indent=4))
    else:
        write_metadata(args.file, summary)


def write_metadata(file, summary):
    """FILE.txt["analysis_result"] = summary, merged into an existing sidecar
    (src/analyse.py:454-468)."""
    meta_path = Path(file).with_suffix(".txt")
    logging.info("Writing metadata to %s", meta_path)
    metadata = {}
    if meta_path.exists():
        with meta_path.open("r") as f:
            metadata = json.load(f)
    metadata["analysis_result"] = summary
    with meta_path.open("w") as f:
        json.dump(metadata, f, sort_keys=True, indent=4)


def cli():
    try:
        main()
    except Exception:
        logging.error("Terminated with error", exc_info=True)
        sys.exit(1)


if __name__ == "__main__":
    cli()
