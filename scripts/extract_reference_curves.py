"""Recover the plotted data series from the reference's matplotlib PDFs.

Several reference results exist only as figures (e.g. the MNIST 1->7 poisoning runs,
``eval/eval_poison/mnist_poison_30_100_AR.pdf``; there is no parsed CSV for them).  matplotlib's PDF
backend writes each line as a FlateDecode content stream of ``x y m`` / ``x y l`` path operators in
page coordinates, and each tick as a short path followed by its text label.  This script

  1. inflates the page content stream (zlib; nothing is executed),
  2. reads the x/y tick marks and their numeric labels -> an affine page->data map per axis,
  3. collects every stroked polyline with more than `min_points` vertices, with its stroke colour
     and dash pattern,
  4. matches each series to a legend entry (legend samples are 2-point lines with the same style,
     followed by the label text),

and writes JSON: {file: {"xlabel", "ylabel", "series": [{"label", "x", "y"}]}}.

    python scripts/extract_reference_curves.py /root/reference/eval/eval_poison/*.pdf -o out.json
"""
from __future__ import annotations

import argparse
import json
import re
import sys
import zlib


def _content_streams(data: bytes) -> list[str]:
    out = []
    for s in re.findall(rb"stream\r?\n(.*?)\r?\nendstream", data, re.S):
        try:
            txt = zlib.decompress(s).decode("latin1")
        except zlib.error:
            continue
        if " Tj" in txt and " l\n" in txt:
            out.append(txt)
    return out


_NUM = r"-?\d+(?:\.\d+)?"


def _parse(txt: str):
    """Token walk: returns (paths, texts).  paths: list of dict(points, color, dash, width);
    texts: list of (x, y, string, angle_is_vertical)."""
    paths, texts = [], []
    color, dash, width = "0 G", "[ ] 0", 1.0
    cur: list[tuple[float, float]] = []
    lines = txt.split("\n")
    i = 0
    td_pos = None
    vertical = False
    while i < len(lines):
        ln = lines[i].strip()
        i += 1
        if not ln:
            continue
        m = re.fullmatch(rf"({_NUM}) ({_NUM}) m", ln)
        if m:
            cur = [(float(m.group(1)), float(m.group(2)))]
            continue
        m = re.fullmatch(rf"({_NUM}) ({_NUM}) l", ln)
        if m:
            cur.append((float(m.group(1)), float(m.group(2))))
            continue
        if ln in ("S", "B") or ln.endswith(" S"):
            if cur:
                paths.append({"points": cur, "color": color, "dash": dash, "width": width})
            cur = []
            continue
        # style operators (may share a line with others)
        for mm in re.finditer(rf"({_NUM}) ({_NUM}) ({_NUM}) RG", ln):
            color = f"{mm.group(1)} {mm.group(2)} {mm.group(3)} RG"
        for mm in re.finditer(rf"(?<![\d.])({_NUM}) G(?![a-z])", ln):
            if " RG" not in ln:
                color = f"{mm.group(1)} G"
        for mm in re.finditer(r"(\[[^\]]*\]) (\d+(?:\.\d+)?) d", ln):
            dash = f"{mm.group(1)} {mm.group(2)}"
        for mm in re.finditer(rf"({_NUM}) w", ln):
            width = float(mm.group(1))
        if ln.startswith("BT"):
            td_pos, vertical = None, False
            mm = re.search(rf"({_NUM}) ({_NUM}) Td", ln)
            if mm:
                td_pos = (float(mm.group(1)), float(mm.group(2)))
            mm = re.search(rf"0 1 -1 0 ({_NUM}) ({_NUM}) Tm", ln)
            if mm:
                td_pos, vertical = (float(mm.group(1)), float(mm.group(2))), True
            # the text may sit on following lines until ET
            block = ln
            while "ET" not in block.split() and i < len(lines):
                block += " " + lines[i].strip()
                i += 1
            mm = re.search(rf"0 1 -1 0 ({_NUM}) ({_NUM}) Tm", block)
            if mm:
                td_pos, vertical = (float(mm.group(1)), float(mm.group(2))), True
            if td_pos is None:
                mm = re.search(rf"({_NUM}) ({_NUM}) Td", block)
                if mm:
                    td_pos = (float(mm.group(1)), float(mm.group(2)))
            s = "".join(re.findall(r"\(((?:[^()\\]|\\.)*)\) Tj", block))
            if s and td_pos is not None:
                texts.append((td_pos[0], td_pos[1], s, vertical))
    return paths, texts


def _num(s: str):
    s = s.replace("\\055", "-").replace("\\u2212", "-").replace("−", "-").strip()
    try:
        return float(s)
    except ValueError:
        return None


def _axis_maps(paths, texts):
    """Tick marks are 2-point paths of length ~3.5 (matplotlib default).  x ticks are vertical
    segments below the axes; y ticks horizontal segments left of them.  Each tick is paired with
    the numeric text label nearest to it."""
    xt, yt = [], []
    for p in paths:
        pts = p["points"]
        if len(pts) != 2:
            continue
        (x0, y0), (x1, y1) = pts
        if abs(x0 - x1) < 1e-6 and 2.0 < abs(y0 - y1) < 5.0:
            xt.append((x0, max(y0, y1)))
        elif abs(y0 - y1) < 1e-6 and 2.0 < abs(x0 - x1) < 5.0:
            yt.append((max(x0, x1), y0))
    nums = [(x, y, _num(s)) for x, y, s, v in texts if not v and _num(s) is not None]

    def fit(ticks, horiz):
        pairs = []
        for tx, ty in ticks:
            best = None
            for x, y, v in nums:
                d = (abs(y - (ty - 20)) + abs(x - tx) / 8) if horiz else (abs(y - ty) + abs(tx - x) / 8)
                if (x < tx if not horiz else y < ty) and (best is None or d < best[0]):
                    best = (d, v)
            if best:
                pairs.append((tx if horiz else ty, best[1]))
        pairs = sorted(set(pairs))
        if len(pairs) < 2:
            return None
        (p0, v0), (p1, v1) = pairs[0], pairs[-1]
        if p1 == p0:
            return None
        a = (v1 - v0) / (p1 - p0)
        return lambda p: v0 + a * (p - p0)

    # keep only ticks that sit on the majority baseline / left edge
    if xt:
        base = max(set(round(t[1], 2) for t in xt), key=lambda b: sum(1 for t in xt if round(t[1], 2) == b))
        xt = [t for t in xt if round(t[1], 2) == base]
    if yt:
        edge = max(set(round(t[0], 2) for t in yt), key=lambda b: sum(1 for t in yt if round(t[0], 2) == b))
        yt = [t for t in yt if round(t[0], 2) == edge]
    return fit(xt, True), fit(yt, False)


def extract(path: str, min_points: int = 8) -> dict:
    data = open(path, "rb").read()
    res = {"series": []}
    for txt in _content_streams(data):
        paths, texts = _parse(txt)
        fx, fy = _axis_maps(paths, texts)
        if fx is None or fy is None:
            continue
        labels = [(x, y, s) for x, y, s, v in texts if not v and _num(s) is None]
        res["xlabel"] = next((s for x, y, s, v in texts if not v and _num(s) is None and y < 20), None)
        res["ylabel"] = next((s for x, y, s, v in texts if v), None)
        # legend samples: 2-point horizontal lines with a label text right of them
        legend = []
        for p in paths:
            pts = p["points"]
            if len(pts) == 2 and abs(pts[0][1] - pts[1][1]) < 1e-6 and abs(pts[1][0] - pts[0][0]) > 20:
                y = pts[0][1]
                cand = [(abs(ty - (y - 6.3)) + abs(tx - pts[1][0]) / 10, s) for tx, ty, s in labels
                        if tx > pts[1][0] and abs(ty - y) < 15]
                if cand:
                    legend.append(((p["color"], p["dash"]), min(cand)[1]))
        for p in paths:
            if len(p["points"]) < min_points:
                continue
            key = (p["color"], p["dash"])
            lab = next((s for k, s in legend if k == key), None)
            res["series"].append({"label": lab, "style": f"{p['color']} dash={p['dash']}",
                                  "x": [round(fx(x), 4) for x, _ in p["points"]],
                                  "y": [round(fy(y), 5) for _, y in p["points"]]})
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("pdfs", nargs="+")
    ap.add_argument("-o", "--out", default=None)
    ap.add_argument("--min-points", type=int, default=8)
    a = ap.parse_args(argv)
    out = {}
    for f in a.pdfs:
        try:
            out[f] = extract(f, a.min_points)
        except Exception as e:  # a figure this parser does not understand is reported, not fatal
            out[f] = {"error": repr(e)}
    js = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(js)
    else:
        sys.stdout.write(js + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
