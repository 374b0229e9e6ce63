"""The README's round-5 and round-6 measurement tables are recomputable from
committed profiles: every row equals what tools/hyg_summary.py derives from
profiles/r0N/hyg/<config>/ (the bench line and the rocprofv3 kernel trace of
the same run).  CPU only."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# README section title -> (profiles directory, rows at least)
TABLES = {"## Round 6: every line": ("r06", 13), "## Round 5": ("r05", 11)}


def readme_rows(title):
    text = open(os.path.join(ROOT, "README.md")).read()
    sec = text[text.index(title):]
    sec = sec[:sec.find("\n## ", 1)] if "\n## " in sec[1:] else sec
    rows = {}
    for ln in sec.splitlines():
        if not ln.startswith("| "):
            continue
        cells = [c.strip() for c in ln.strip("|").split("|")]
        if len(cells) != 8 or cells[0] == "config":
            continue
        rows[cells[0].split()[0]] = cells
    return rows


@pytest.mark.parametrize("title", sorted(TABLES))
def test_readme_table_matches_profiles(title):
    rnd, least = TABLES[title]
    hyg = os.path.join(ROOT, "profiles", rnd, "hyg")
    if not os.path.isdir(hyg):
        pytest.skip(f"no {rnd} profiles")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "hyg_summary.py"), hyg],
                         capture_output=True, text=True, check=True).stdout
    got = {r["cfg"]: r for r in map(json.loads, out.splitlines())}
    rows = readme_rows(title)
    assert len(rows) >= least, sorted(rows)
    for cfg, c in rows.items():
        r = got[cfg]
        assert c[1] == f"`{r['kernel']}`", cfg
        assert float(c[2]) == r["Gkeys_s"], cfg
        assert float(c[3]) == r["frac_event"], cfg
        assert float(c[4]) == r["frac_trace"], cfg
        if c[5] != "—":
            assert float(c[5]) == round(r["read_only_GBps"] / 8000.0, 4), cfg
        assert c[6] == r["parity"] == "ok", cfg
        assert float(c[7]) == r["cpu"], cfg
        # the event-timed and the trace-derived figure of one run agree
        assert abs(r["event_over_trace"] - 1) < 0.02, (cfg, r["event_over_trace"])
