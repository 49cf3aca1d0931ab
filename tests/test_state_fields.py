"""The C-ABI state packer (dk_fdo_from_fields / dk_do_from_fields, SURVEY.md §8(b) "State
wire format"): a caller's FdoState / DoState fields -> the 128-B wire format.  Host-only
functions of libdoko_amd.so, so this runs without a GPU.

The oracle fills the fields from its own restatement of FdoState / DoState (the fields of
rs-full-doko/src/state/state.rs:24-75 and rs-doko/src/state/state.rs:28-76) along random
games through every phase (reservations including weddings and solos, announcement rounds,
finished games) and along the four reference full-game traces; the library's packing must
equal the oracle's own packing byte for byte, and packing must invert dk_*_to_fields."""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle_lib as ol
from test_gpu_parity import do_states, fdo_states

import master_doko_reinforcement_learning_amd as dk

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _oracle_fdo_fields(s):
    f = dk.FdoFields()
    ol.lib().or_fdo_fields(ctypes.c_void_p(s.h), ctypes.byref(f))
    return f


def _oracle_do_fields(s):
    f = dk.DoFields()
    ol.lib().or_do_fields(ctypes.c_void_p(s.h), ctypes.byref(f))
    return f


def _trace_states():
    """Every state along the four reference traces (state.rs:551-1808), replayed like
    test_oracle_golden.test_fdo_full_game_trace (forced passes inserted as the rules demand)."""
    from test_oracle_golden import _meaningful_steps, hand_bits
    with open(os.path.join(GOLD, "fdo_traces.json")) as fh:
        games = json.load(fh)
    out = []
    kind = lambda a: 2 if a <= 23 else (0 if a <= 32 else 1)
    for g in games:
        s = ol.FdoState.from_hands([hand_bits(h) for h in g["hands"]], g["start_player"])
        out.append(s.clone())
        for p, a, _, _ in _meaningful_steps(g):
            while s.info()["phase"] == 1 and not (kind(a) == 1 and s.info()["current_player"] == p):
                s.play(38)
                out.append(s.clone())
            s.play(a)
            out.append(s.clone())
    return out


def test_fdo_from_fields_equals_oracle_pack():
    states = fdo_states(24, 41) + _trace_states()
    kinds = set()
    for s in states:
        f = _oracle_fdo_fields(s)
        kinds.add((f.phase, f.rr_kind, f.team_kind))
        got = dk.fdo_from_fields(f)
        assert got == s.pack()
        back = dk.fdo_to_fields(got)
        assert back.ann_n == f.ann_n
        # the occurrence list is not part of the wire format: restore it, then the rest must invert
        for k in range(12):
            back.ann_card_index[k], back.ann_player[k], back.ann_announcement[k] = \
                f.ann_card_index[k], f.ann_player[k], f.ann_announcement[k]
        assert dk.fdo_from_fields(back) == got
    assert len(kinds) >= 6, kinds     # phases x reservation results x team states covered


def test_do_from_fields_equals_oracle_pack():
    for s in do_states(24, 43):
        f = _oracle_do_fields(s)
        got = dk.do_from_fields(f)
        assert got == s.pack()
        assert dk.do_from_fields(dk.do_to_fields(got)) == got


def test_from_fields_rejects_inconsistent_fields():
    s = fdo_states(2, 7)[30]
    f = _oracle_fdo_fields(s)
    bad = dk.FdoFields.from_buffer_copy(f)
    bad.hands[0] |= bad.hands[1]                       # a third copy of some card
    with pytest.raises(dk.DokoError):
        dk.fdo_from_fields(bad)
    bad = dk.FdoFields.from_buffer_copy(f)
    bad.card_index += 1                               # card_index against the tricks
    with pytest.raises(dk.DokoError):
        dk.fdo_from_fields(bad)
    bad = dk.FdoFields.from_buffer_copy(f)
    bad.game_type = 9
    with pytest.raises(dk.DokoError):
        dk.fdo_from_fields(bad)
    from master_doko_reinforcement_learning_amd import _native
    assert _native.lib().dk_fdo_from_fields(None, None) == -1
