"""Copy the bench JSON lines (and test summaries) of a gpurun output directory into profiles/ (tracked):

    python scripts/keep_results.py gpurun_out/r6a profiles/r6/a

Each OUT/NAME.txt with a bench JSON line becomes DEST/NAME.json (the line, pretty-printed); tests.txt / smoke.txt
keep their last lines; the runner's one-line summaries are collected in DEST/summary.txt."""
import json
import sys
from pathlib import Path


def main(src: str, dst: str) -> None:
    s, d = Path(src), Path(dst)
    d.mkdir(parents=True, exist_ok=True)
    summary = []
    for f in sorted(s.glob("*.txt")):
        lines = f.read_text(errors="replace").splitlines()
        js = [ln for ln in lines if ln.startswith("{")]
        if js:
            try:
                rec = json.loads(js[-1])
            except ValueError:
                continue
            (d / (f.stem + ".json")).write_text(json.dumps(rec, indent=1) + "\n")
            w = rec.get("round_wall_ms") or []
            med = sorted(w)[len(w) // 2] if w else None
            summary.append(f"{f.stem}: ms/round {rec.get('ms_per_step'):.4f} median {med} "
                           f"final_acc {rec.get('final_test_acc')} contributors/block {rec.get('contributors_per_block')}")
        elif f.stem.startswith(("tests", "test_", "smoke")):
            tail = [ln for ln in lines if ln.strip()][-3:]
            # (a test step's file is named after its -k expression: no spaces in the kept name)
            (d / f.name.replace(" ", "_")).write_text("\n".join(tail) + "\n")
            summary.append(f"{f.stem}: {tail[-1] if tail else ''}")
    (d / "summary.txt").write_text("\n".join(summary) + "\n")
    print("\n".join(summary))


if __name__ == "__main__":
    main(*sys.argv[1:3])
