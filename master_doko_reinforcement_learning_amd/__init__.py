"""MI355X-native determinized-MCTS rollout engine for Doppelkopf.

The hot path of theodm/master_doko_reinforcement_learning (rs-doko-mcts UCT over
rs-full-doko / rs-doko rules, CAP and rule-based determinization, policy fusion) as HIP kernels
for gfx950 behind the C-ABI of include/doko_amd.h.  See DESIGN.md.
"""
from . import _native
from .api import (AR_CONSISTENT, AR_NOT_CONSISTENT, AR_PANIC, FUSE_AVG, FUSE_MAXN, GAME_DOKO, GAME_FULL_DOKO, GAME_TTT,
                  NOT_CONSISTENT_REASONS, NUM_ACTIONS, AlphaZeroSearch, ArImpiPolicy, ARSampling, CachedMCTS, DefaultImpiPolicy,
                  DokoError, Engine, McEnv, PolicyFusionAverageStrategy, PolicyFusionMaxN, SmallRng,
                  card_matching_full, sample_assignment_full, splitmix_rng_states, az_encode, az_records, az_step,
                  FdoFields, DoFields, fdo_from_fields, fdo_to_fields, do_from_fields, do_to_fields,
                  ttt_state, tic_tac_toe_player, tic_tac_toe_games, sample_interleaved)

__all__ = ["Engine", "McEnv", "CachedMCTS", "SmallRng", "card_matching_full", "sample_assignment_full", "PolicyFusionMaxN", "PolicyFusionAverageStrategy",
           "DefaultImpiPolicy", "AlphaZeroSearch", "DokoError", "splitmix_rng_states", "GAME_FULL_DOKO", "GAME_DOKO", "GAME_TTT",
           "FUSE_MAXN", "FUSE_AVG", "NUM_ACTIONS", "az_records", "az_step", "az_encode", "ARSampling", "ArImpiPolicy", "AR_CONSISTENT",
           "AR_NOT_CONSISTENT", "AR_PANIC", "sample_interleaved", "NOT_CONSISTENT_REASONS", "build", "FdoFields", "DoFields",
           "fdo_from_fields", "fdo_to_fields", "do_from_fields", "do_to_fields", "ttt_state",
           "tic_tac_toe_player", "tic_tac_toe_games"]


def build(verbose=False):
    return _native.build(verbose=verbose)
