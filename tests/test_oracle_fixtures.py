"""The committed ORACLE regression fixtures (tests/golden/make_oracle_fixtures.py, SURVEY.md
§8(c)) are reproduced by the current oracle: a drifting restatement fails here before any
GPU comparison against it.  CPU only."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_oracle_fixtures as mk  # noqa: E402


def _load(name):
    with open(os.path.join(HERE, "golden", name)) as fh:
        return json.load(fh)


def test_oracle_rollouts_fixture():
    want = _load("oracle_rollouts.json")
    assert len(want) == 1000
    assert mk.rollouts(200) == want[:200]


def test_oracle_searches_fixture():
    want = _load("oracle_searches.json")
    assert len(want) == 100
    assert mk.searches(12) == want[:12]


def test_oracle_cap_fixture():
    want = _load("oracle_cap.json")
    assert len(want) == 100 and all(w["consistent"] for w in want)
    assert mk.cap(100) == want
