/*
 * doko_amd.h — C-ABI of the MI355X determinized-MCTS rollout engine.
 *
 * This is the drop-in boundary for the hot path of
 * theodm/master_doko_reinforcement_learning.  Every entry
 * point names the Rust interface it replaces.  Plain pointers and sizes only;
 * no torch / HIP types in the signatures.  All compute runs on the GPU: the
 * library has no CPU fallback and returns DK_E_NO_DEVICE when no gfx950
 * device is usable.
 *
 * Two flavours of every batched call:
 *   dk_xxx(...)        host pointers; the call copies in/out and synchronises.
 *   dk_xxx_async(...)  device pointers + an opaque stream handle (hipStream_t);
 *                      nothing is synchronised.  NULL selects the context's own
 *                      non-blocking stream, which is NOT ordered after work queued
 *                      on the legacy default stream: pass the caller's stream.
 *
 * Reference interfaces (file:line under /root/reference):
 *   McEnvState trait ......... rs-doko-mcts/src/env/env_state.rs:7-28
 *   McFullDokoEnvState ....... rs-doko-mcts/src/env/envs/env_state_full_doko.rs:22-220
 *   McDokoEnvState ........... rs-doko-mcts/src/env/envs/env_state_doko.rs:15-170
 *   TicTacToe McEnvState ..... rs-doko-mcts/src/example/tic_tac_toe_impl.rs:17-63
 *   CachedMCTS ............... rs-doko-mcts/src/mcts/mcts.rs:252-321
 *   EvFullDokoMCTSPolicy ..... rs-doko-evaluator/src/full_doko/policy/mcts_policy.rs:136-169
 *   SamplingFn / CAPSampling . rs-doko-py-bridge/src/compare_impi/compare_impi.rs:49-82
 *   PolicyFusionFn ........... rs-doko-py-bridge/src/compare_impi/policy_fusion.rs:9-123
 *   DefaultImpiPolicy ........ rs-doko-py-bridge/src/compare_impi/compare_impi.rs:212-371
 *   FdoState::new_game ....... rs-full-doko/src/state/state.rs:165-176
 *   DoState::new_game ........ rs-doko/src/state/state.rs:159-168
 */
#ifndef DOKO_AMD_H
#define DOKO_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DK_ABI_VERSION 1
#define DK_STATE_BYTES 128
#define DK_NUM_ACTIONS 39 /* FdoAction::COUNT (rs-full-doko/src/action/action.rs:9-54) */
#define DK_NONE 0xFF

/* ---- games ---------------------------------------------------------------- */
enum dk_game {
    DK_GAME_FULL_DOKO = 0, /* rs-full-doko: 39 actions, solos, announcements, DKV scoring */
    DK_GAME_DOKO = 1,      /* rs-doko: 26 actions (bits 0-25 == FdoAction bits 0-25)      */
    DK_GAME_TTT = 2        /* tic-tac-toe of rs-doko-mcts/src/example: actions 0-8         */
};

/* ---- status codes (the Rust path panics instead) -------------------------- */
enum dk_status {
    DK_OK = 0,
    DK_E_INVALID = -1,   /* bad argument / unknown game / sizes                        */
    DK_E_CAPACITY = -2,  /* node pool or batch larger than the context was created for */
    DK_E_STATE = -3,     /* illegal action for a state, or a malformed state           */
    DK_E_NO_DEVICE = -4, /* no usable gfx950 device / HIP error                        */
    DK_E_LAUNCH = -5     /* kernel launch or execution failure                         */
};

/* ---- packed states (128 bytes; byte 127 is the game tag) ------------------
 * Hands use the reference bit layout (rs-full-doko/src/hand/hand.rs:17-20):
 * bit k (0..23) = first copy of card kind k, bit k+24 = second copy; card kind
 * order = FdoCard (♦9 ♦10 ♦J ♦Q ♦K ♦A ♥… ♣… ♠…).  Players 0..3 = BOTTOM LEFT TOP RIGHT.
 */
typedef struct dk_fdo_state {
    uint64_t hands[4];       /*   0: FdoState.hands                                         */
    uint8_t cards[48];       /*  32: card kind played at card index i (DK_NONE = not yet)   */
    uint8_t eyes[4];         /*  80: player_eyes (<= 240)                                   */
    uint8_t ntricks[4];      /*  84: player_num_tricks                                      */
    uint32_t trick_winners;  /*  88: 2 bits per completed trick (trick t at bits 2t..2t+1)   */
    uint8_t res[4];          /*  92: played reservations in round order (FdoReservation)    */
    uint8_t res_start;       /*  96: reservation round starting player                      */
    uint8_t res_len;         /*  97                                                          */
    uint8_t card_index;      /*  98                                                          */
    uint8_t phase;           /*  99: 0 Reservation 1 Announcement 2 PlayCard 3 Finished     */
    uint8_t current_player;  /* 100: DK_NONE when finished                                  */
    uint8_t game_type;       /* 101: FdoGameType or DK_NONE                                 */
    uint8_t rr_kind;         /* 102: reservation result: DK_NONE, 0 none, 1 solo, 2 wedding */
    uint8_t rr_player;       /* 103                                                          */
    uint8_t rr_reservation;  /* 104: FdoReservation of the winning solo                     */
    uint8_t team_kind;       /* 105: 0 InReservations 1 WeddingUnsolved 2 WeddingSolved 3 NoWedding */
    uint8_t wedding_player;  /* 106                                                          */
    uint8_t solved_trick;    /* 107: WeddingSolved.solved_trick_index                       */
    uint8_t re_players;      /* 108: bit mask                                               */
    uint8_t re_lowest;       /* 109: FdoAnnouncement bit (1,2,4,8,16,32) or 0 = None        */
    uint8_t contra_lowest;   /* 110                                                          */
    uint8_t ann_turns;       /* 111: number_of_turns_without_announcement                   */
    uint8_t ann_start;       /* 112: starting player of the announcement round             */
    uint8_t ann_allowed;     /* 113: current_player_allowed_announcements (FdoAnnouncementSet) */
    uint8_t ann_count;       /* 114: announcement occurrences recorded (<= 12)             */
    uint8_t ann_players;     /* 115: mask of players that made an announcement             */
    uint8_t n_tricks;        /* 116: tricks started (FdoState.tricks.len())                 */
    uint8_t reserved[10];    /* 117                                                          */
    uint8_t game;            /* 127: DK_GAME_FULL_DOKO                                      */
} dk_fdo_state;

typedef struct dk_do_state {
    uint64_t hands[4];       /*   0: DoState.hands (rs-doko/src/hand/hand.rs:13)            */
    uint8_t cards[48];       /*  32                                                          */
    uint8_t eyes[4];         /*  80                                                          */
    uint8_t ntricks[4];      /*  84                                                          */
    uint32_t trick_winners;  /*  88                                                          */
    uint8_t res[4];          /*  92: DoReservation (0 Wedding, 1 Healthy), DK_NONE empty    */
    uint8_t res_start;       /*  96                                                          */
    uint8_t res_len;         /*  97                                                          */
    uint8_t card_index;      /*  98                                                          */
    uint8_t phase;           /*  99: 0 Reservation 1 PlayCard 2 Finished (DoPhase)          */
    uint8_t current_player;  /* 100                                                          */
    uint8_t rr_kind;         /* 101: DK_NONE, 0 NoReservation, 2 Wedding                    */
    uint8_t rr_player;       /* 102                                                          */
    uint8_t team_kind;       /* 103                                                          */
    uint8_t wedding_player;  /* 104                                                          */
    uint8_t solved_trick;    /* 105                                                          */
    uint8_t re_players;      /* 106                                                          */
    uint8_t trick_index;     /* 107: current_trick_index                                    */
    uint8_t reserved[19];    /* 108                                                          */
    uint8_t game;            /* 127: DK_GAME_DOKO                                           */
} dk_do_state;

typedef struct dk_ttt_state {
    uint8_t board[9];        /* 0 empty, 1 X, 2 O                                            */
    uint8_t finish;          /* 0 NotFinished 1 Xwon 2 Owon 3 Draw                          */
    uint8_t last_action;     /* DK_NONE or cell                                              */
    uint8_t reserved[116];
    uint8_t game;            /* 127: DK_GAME_TTT                                             */
} dk_ttt_state;

typedef union dk_state {
    uint8_t raw[DK_STATE_BYTES];
    dk_fdo_state fdo;
    dk_do_state dk;
    dk_ttt_state ttt;
} dk_state;

/* AlphaZero game record: the packed rs-full-doko state plus its announcement
 * occurrence list (FdoAnnouncements.announcements, announcement/announcement.rs:47-59),
 * which the network's encoder reads (encode_pi.rs:135-170) and dk_fdo_state has no room for.
 * ann_code[k] = player << 4 | (announcement action - 33): 0 ReContra, 1 No90, 2 No60,
 * 3 No30, 4 Black (FdoAction::AnnouncementReContra always records FdoAnnouncement::ReContra,
 * action/action.rs:295-310). */
typedef struct dk_az_state {
    dk_state state;          /*   0                                                          */
    uint8_t ann_card[12];    /* 128: card_index of each occurrence                           */
    uint8_t ann_code[12];    /* 140                                                          */
    uint8_t ann_n;           /* 152                                                          */
    uint8_t reserved[7];     /* 153                                                          */
} dk_az_state;

/* ---- state wire format from the reference's fields (host only, no device) -------
 * dk_fdo_fields mirrors FdoState (rs-full-doko/src/state/state.rs:24-75) field by field,
 * so a caller holding an FdoState fills it without knowing the 128-B layout:
 *   reservations_round  (reservation/reservation_round.rs:9-77)  res_start, res_len, reservations[]
 *                        FdoReservation (reservation/reservation.rs:11-24): 0 Healthy 1 Wedding
 *                        2 DiamondsSolo 3 HeartsSolo 4 SpadesSolo 5 ClubsSolo 6 QueensSolo
 *                        7 JacksSolo 8 TrumplessSolo
 *   tricks              (trick/trick.rs:10-17)  n_tricks, trick_start[], trick_cards[][] (FdoCard or -1)
 *   hands               (hand/hand.rs:17-20)     reference bit layout
 *   announcements       (announcement/announcement.rs:47-59)  the occurrence list (card_index,
 *                        player, FdoAnnouncement bit), lowest Re / Kontra (bit, 0 = None),
 *                        number_of_turns_without_announcement, starting_player,
 *                        current_player_allowed_announcements (FdoAnnouncementSet bits)
 *   card_index, current_player (-1 = None), current_phase (0 Reservation 1 Announcement
 *   2 PlayCard 3 Finished), reservation_result (rr_kind -1 None, 0 NoReservation, 1 Solo,
 *   2 Wedding; rr_player; rr_reservation), game_type (FdoGameType, -1 = None), player_eyes,
 *   player_num_tricks, team_state (team/team_logic.rs:11-28: team_kind 0 InReservations
 *   1 WeddingUnsolved 2 WeddingSolved 3 NoWedding; wedding_player; solved_trick_index;
 *   re_players as a player bit mask).
 * end_of_game_stats is derived (recomputed by dk_env_rewards_batch) and trick winners are
 * recomputed from the cards and the game type.  dk_fdo_to_fields is the inverse except for
 * the announcement occurrence list, which the wire format keeps only as a count and a
 * player mask (ann_card_index / ann_player / ann_announcement come back as -1 / -1 / 0).
 * Returns DK_OK, DK_E_INVALID (NULL) or DK_E_STATE (fields that contradict each other:
 * card counts, card_index against the tricks, players or enums out of range). */
typedef struct dk_fdo_fields {
    uint64_t hands[4];
    uint32_t player_eyes[4];
    uint32_t player_num_tricks[4];
    int8_t res_start;
    int8_t res_len;
    int8_t reservations[4];
    int8_t n_tricks;
    int8_t trick_start[12];
    int8_t trick_cards[12][4];
    int8_t ann_n;
    int8_t ann_card_index[12];
    int8_t ann_player[12];
    uint8_t ann_announcement[12];
    uint8_t re_lowest;
    uint8_t contra_lowest;
    int8_t ann_turns_without;
    int8_t ann_start;
    uint8_t ann_allowed;
    int8_t card_index;
    int8_t current_player;
    int8_t phase;
    int8_t rr_kind;
    int8_t rr_player;
    int8_t rr_reservation;
    int8_t game_type;
    int8_t team_kind;
    int8_t wedding_player;
    int8_t solved_trick;
    uint8_t re_players;
} dk_fdo_fields;

/* dk_do_fields mirrors DoState (rs-doko/src/state/state.rs:28-76): reservations (DoReservation
 * 0 Wedding 1 Healthy, -1 = not yet played, in round order from res_start), tricks (12 slots,
 * present ones with trick_start >= 0; cards -1 when not yet played), hands (bit layout of
 * rs-doko/src/hand/hand.rs:13), current_player (-1 = None), phase (0 Reservation 1 PlayCard
 * 2 Finished), current_trick_index, reservation result (rr_kind -1 None, 0 NoReservation,
 * 2 Wedding; rr_player), player_eyes, player_num_tricks, team_state (teams/team_logic.rs:
 * team_kind, wedding_player, solved_trick, re_players mask). */
typedef struct dk_do_fields {
    uint64_t hands[4];
    uint32_t player_eyes[4];
    uint32_t player_num_tricks[4];
    int8_t res_start;
    int8_t reservations[4];
    int8_t trick_start[12];
    int8_t trick_cards[12][4];
    int8_t current_player;
    int8_t phase;
    int8_t trick_index;
    int8_t rr_kind;
    int8_t rr_player;
    int8_t team_kind;
    int8_t wedding_player;
    int8_t solved_trick;
    uint8_t re_players;
} dk_do_fields;

int dk_fdo_from_fields(const dk_fdo_fields* fields, dk_state* out);
int dk_fdo_to_fields(const dk_state* state, dk_fdo_fields* fields);
int dk_do_from_fields(const dk_do_fields* fields, dk_state* out);
int dk_do_to_fields(const dk_state* state, dk_do_fields* fields);

/* ---- context ---------------------------------------------------------------- */
typedef struct dk_config {
    int32_t device;          /* HIP device ordinal                                          */
    uint32_t max_roots;      /* largest batch of roots one search call may carry            */
    uint32_t max_iterations; /* largest `iterations` one search call may use                */
    uint32_t slot_capacity;  /* child slots per root in the main pools (0 = 64 + 8 x        */
                             /* max_iterations, halved while the pools would take more than */
                             /* half of the free device memory); see dk_pool_high_water     */
} dk_config;

typedef struct dk_ctx dk_ctx;

/* The node / state pools hold min(max_roots, resident roots) trees at once (resident
 * roots = CUs x 12 waves x 64 lanes; env DK_POOL_ROOTS overrides).  The search grid is
 * persistent: a batch larger than the pools streams through them, one wave-sized group of
 * roots at a time, so max_roots bounds the batch, not the memory.
 * Child slots: a search needs at most 42 + 12 x iterations of them (proven bound) but
 * measured far fewer, so the main pools hold slot_capacity per root (default
 * 64 + 8 x max_iterations, rounded up to a multiple of 256; env DK_SLOT_CAPACITY overrides).  A root that runs out is
 * searched again, from its seed, by a second launch over a small pool with the proven
 * bound (4,096 roots at once): results are identical whatever the capacity.  With
 * slot_capacity at or above the proven bound there is no second pool. */
dk_ctx* dk_create(const dk_config* cfg);
void dk_destroy(dk_ctx* ctx);
int dk_last_error(const dk_ctx* ctx);
const char* dk_status_string(int status);
int dk_abi_version(void);

/* ---- game construction ------------------------------------------------------
 * FdoState::new_game(SmallRng::seed_from_u64(seed[i])) / DoState::new_game(...)
 * rs-full-doko/src/state/state.rs:165-176, rs-doko/src/state/state.rs:159-168.
 */
int dk_new_game_batch(dk_ctx* ctx, int game, const uint64_t* seeds, uint32_t n, dk_state* out);
int dk_new_game_batch_async(dk_ctx* ctx, int game, const uint64_t* d_seeds, uint32_t n, dk_state* d_out, void* stream);

/* ---- McEnvState (rs-doko-mcts/src/env/env_state.rs:7-28), batched ----------
 * allowed_actions(first_expansion) -> FdoAllowedActions bits (u64 per state)
 * by_action(action)                -> state stepped in place (one-hot action bit)
 * rewards_or_none()                -> has_rewards[i] and rewards[4*i..]
 * random_rollout(rng)              -> rewards[4*i..] ; rng[4*i..] = Xoshiro256++ state, advanced
 */
int dk_env_allowed_batch(dk_ctx* ctx, const dk_state* states, uint32_t n, int first_expansion, uint64_t* masks);
int dk_env_step_batch(dk_ctx* ctx, dk_state* states, const uint64_t* action_bits, uint32_t n);
int dk_env_rewards_batch(dk_ctx* ctx, const dk_state* states, uint32_t n, int32_t* has_rewards, double* rewards);
int dk_env_rollout_batch(dk_ctx* ctx, const dk_state* states, uint64_t* rng_states, uint32_t n, double* rewards);
int dk_env_rollout_batch_async(dk_ctx* ctx, const dk_state* d_states, uint64_t* d_rng_states, uint32_t n,
                               double* d_rewards, void* stream);
/* random_action_for_current_player_no_announcement applied k[i] times
 * (rs-full-doko/src/state/state.rs:401-431; rs-doko uses random_action_for_current_player). */
int dk_env_random_plies_batch(dk_ctx* ctx, dk_state* states, uint64_t* rng_states, const uint32_t* plies, uint32_t n);
int dk_env_random_plies_batch_async(dk_ctx* ctx, dk_state* d_states, uint64_t* d_rng_states, const uint32_t* d_plies,
                                    uint32_t n, void* stream);
int dk_env_step_batch_async(dk_ctx* ctx, dk_state* d_states, const uint64_t* d_action_bits, uint32_t n, void* stream);
/* observation.allowed_actions_current_player (legal set incl. announcements), state.rs:434-481 */
int dk_legal_actions_async(dk_ctx* ctx, const dk_state* d_states, uint32_t n, uint64_t* d_masks, void* stream);

/* ---- CachedMCTS::monte_carlo_tree_search (rs-doko-mcts/src/mcts/mcts.rs:284-315)
 * One independent UCT search per root (the reference's sequential per-root
 * semantics; parallel only across roots).  rng seed: SmallRng::seed_from_u64(seeds[i]).
 * visits/values: [n][39] by action index (mcts_policy.rs:95-104, values as f64
 * win_score/visits); best[i] = max_by_key(visits) over root children in
 * expansion order (last maximum wins), DK_NONE when the root has no children.
 * `c` is the UCT exploration constant as f64 (the evaluator passes (double)(float)c).
 */
int dk_search_batch(dk_ctx* ctx, int game, const dk_state* roots, const uint64_t* seeds, uint32_t n,
                    uint32_t iterations, double c, uint32_t* visits, double* values, uint8_t* best);
int dk_search_batch_async(dk_ctx* ctx, int game, const dk_state* d_roots, const uint64_t* d_seeds, uint32_t n,
                          uint32_t iterations, double c, uint32_t* d_visits, double* d_values, uint8_t* d_best,
                          void* stream);
/* The same search continuing the caller's SmallRng: CachedMCTS::monte_carlo_tree_search(state, c,
 * iterations, random: &mut SmallRng) (rs-doko-mcts/src/mcts/mcts.rs:294-315), whose callers thread
 * one stream through many searches (rs-doko-mcts/src/example/tic_tac_toe_player.rs:9-36 uses one
 * seed_from_u64(999) stream for every move of 1000 games).  rng_states[4*i .. 4*i+3] is root i's
 * Xoshiro256++ state (s0..s3); on return it holds the state after the search, which has consumed
 * exactly what the reference consumes: every expansion's random_single and every rollout, then one
 * u64 for the final random_bool((1f32/1000f32) as f64) (mcts.rs:231).  A root that fails (DK_E_STATE)
 * keeps its input state. */
int dk_search_batch_rng(dk_ctx* ctx, int game, const dk_state* roots, uint64_t* rng_states, uint32_t n,
                        uint32_t iterations, double c, uint32_t* visits, double* values, uint8_t* best);
int dk_search_batch_rng_async(dk_ctx* ctx, int game, const dk_state* d_roots, uint64_t* d_rng_states, uint32_t n,
                              uint32_t iterations, double c, uint32_t* d_visits, double* d_values, uint8_t* d_best,
                              void* stream);

/* ---- determinization: SamplingFn::sample ------------------------------------
 * out[i*samples + s] = sample(infostates[i], SmallRng::seed_from_u64(seeds[i*samples+s])), by game:
 *   DK_GAME_FULL_DOKO: CAPSampling -> card_matching_full
 *       (compare_impi.rs:64-81 -> rs-full-doko/src/matching/card_matching.rs:469-497)
 *   DK_GAME_DOKO:      sample_assignment_full(state, &state.observation_for_current_player(), rng)
 *       (rs-doko-assignment/src/assignment.rs:472-580; observation rs-doko/src/state/state.rs:336-410)
 * Any other game, or a finished rs-full-doko infostate, is DK_E_STATE. An rs-doko
 * infostate on which the reference sampler panics (a hidden card that no player
 * with open slots may hold, assignment.rs:430-433) is DK_E_STATE as well.
 */
int dk_determinize_batch(dk_ctx* ctx, const dk_state* infostates, uint32_t n_info, uint32_t samples,
                         const uint64_t* seeds, dk_state* out);
int dk_determinize_batch_async(dk_ctx* ctx, const dk_state* d_infostates, uint32_t n_info, uint32_t samples,
                               const uint64_t* d_seeds, dk_state* d_out, void* stream);

/* ---- PolicyFusionFn::fuse (policy_fusion.rs:23-123) --------------------------
 * mode DK_FUSE_MAXN: per infostate sum of per-sample visit ranks (u32) -> first
 *   minimum, disallowed actions ranked UINT32_MAX.  acc_u32 = [n_info][39] rank
 *   sums (0 for disallowed actions, so partial sums add across ranks).
 * mode DK_FUSE_AVG: per infostate sum over samples of visits/total (f32) -> last
 *   maximum.                           acc_f32 = [n_info][39] probability sums.
 * The _accumulate/_select split lets a multi-GPU caller all-reduce(sum) the
 * accumulators between the two steps (RCCL over xGMI).
 */
enum dk_fuse_mode { DK_FUSE_MAXN = 0, DK_FUSE_AVG = 1 };
int dk_fuse(dk_ctx* ctx, const uint32_t* visits, uint32_t n_info, uint32_t samples, const uint64_t* allowed,
            int mode, uint8_t* action);
int dk_fuse_accumulate_async(dk_ctx* ctx, const uint32_t* d_visits, uint32_t n_info, uint32_t samples,
                             const uint64_t* d_allowed, int mode, uint32_t* d_acc_u32, float* d_acc_f32, void* stream);
/* dk_fuse_accumulate_async with per-sample flags d_valid[n_info * samples]: samples with 0
 * (failed determinizations, compare_impi.rs:276-288) take no part in the fusion. */
int dk_fuse_accumulate_masked_async(dk_ctx* ctx, const uint32_t* d_visits, uint32_t n_info, uint32_t samples,
                                    const uint8_t* d_valid, const uint64_t* d_allowed, int mode, uint32_t* d_acc_u32,
                                    float* d_acc_f32, void* stream);
int dk_fuse_select_async(dk_ctx* ctx, uint32_t n_info, int mode, const uint64_t* d_allowed, const uint32_t* d_acc_u32,
                         const float* d_acc_f32, uint8_t* d_action, void* stream);

/* ---- DefaultImpiPolicy::execute (compare_impi.rs:212-371), batched ----------
 * For each infostate: `samples` CAP determinizations -> one UCT search each ->
 * fusion. actions[i] = fused action; visits [n_info*samples][39] optional (NULL).
 */
int dk_decide_batch(dk_ctx* ctx, const dk_state* infostates, uint32_t n_info, uint32_t samples,
                    const uint64_t* seeds, uint32_t iterations, double c, int fuse_mode, uint8_t* actions,
                    uint32_t* visits);

/* ---- AlphaZero PUCT search: mcts_search (rs-doko-alpha-zero/src/alpha_zero/mcts/async_mcts.rs:224-406)
 * over FdoAzEnvState (rs-doko-alpha-zero/src/env/envs/full_doko/full_doko.rs:15-172), batched over
 * n_games independent games.  The reference awaits its batch processor (the network) once for the
 * root and once per iteration; here the caller runs the network between the launches, on the
 * same stream, over the leaf records (dk_az_state) the search writes:
 *
 *   dk_az_begin_async   roots (dk_az_state records) -> d_eval[g] = root  (new_root_node, node.rs:209-244)
 *   network(d_eval)     -> value[n][4] (POV of each state's current player), logits[n][39]
 *   dk_az_root_async    priors = softmax(logits) mixed with the root's Dirichlet noise (1 - eps, eps),
 *                       restricted to the root's allowed actions and renormalised; announcements are
 *                       offered at the root iff epoch >= 10.  d_noise == NULL (the reference's way):
 *                       each game draws Dirichlet([dirichlet_alpha; 39]) from its own SmallRng
 *                       (rand_distr 0.5.1, async_mcts.rs:111-113; alpha > 0 and finite, as the
 *                       crate requires: alpha <= 0.1 takes its Beta stick-breaking construction,
 *                       larger alphas its Gamma one); otherwise d_noise[n][39] is used and nothing
 *                       is drawn
 *                                                                        (expand_root_node, async_mcts.rs:71-196)
 *   repeat `iterations` times:
 *     dk_az_select_async  PUCT descent, leaf expansion; d_eval[g] = leaf state,
 *                         d_need_eval[g] = 0 for a terminal leaf (its network row is ignored)
 *                                                                        (mcts.rs:23-74, 306-420)
 *     network(d_eval)
 *     dk_az_backup_async  leaf priors = softmax over its allowed actions' logits; backpropagate
 *                         the value (or the terminal rewards player_points/8)  (async_mcts.rs:280-345, mcts.rs:250-280)
 *   dk_az_finish_async  random_bool(1/5000), then select_action: temperature_mode 0 = None
 *                       (greedy, last maximum), 1 = infinite (uniform), 2 = finite `temperature`
 *                       (visits^(1/T) WeightedIndex); d_visits[n][39] = root child visits
 *                                                                        (async_mcts.rs:347-405, mcts.rs:185-248)
 * seeds[g] seeds game g's SmallRng: the root noise first, then the final draws.
 *   dk_az_rng_async     set = 1 (between begin and root): game g continues the SmallRng state
 *                       d_rng[g][4] (Xoshiro256++ words) instead of seeds[g], like the reference's
 *                       `rng: &mut SmallRng` carried across searches; set = 0 (any time after begin):
 *                       d_rng[g][4] = game g's current state (after finish: the stream's end state)
 * One AZ search batch per context at a time; node/state pools grow on demand (48 B per node,
 * 1 + 12 (iterations + 1) + 39 nodes and iterations + 2 packed states per game).
 */
int dk_az_begin_async(dk_ctx* ctx, const dk_az_state* d_roots, const uint64_t* d_seeds, uint32_t n_games,
                      uint32_t iterations, int epoch, dk_az_state* d_eval, void* stream);
int dk_az_root_async(dk_ctx* ctx, const float* d_value, const float* d_logits, const float* d_noise, float dirichlet_alpha,
                     float dirichlet_epsilon, void* stream);
int dk_az_rng_async(dk_ctx* ctx, uint64_t* d_rng, int set, void* stream);
/* glibc's logf (fn 0) / expf (fn 1) as the device computes them for the root noise's Beta draws
 * (engine/libm_f32.h; Rust's f32::ln / f32::exp call the platform libm): d_y[i] = fn(x_i) for the
 * f32 whose bits are first + i * stride (mod 2^32), i < n.  Exported so that the restatement can be
 * checked against the host's glibc across the whole f32 range (tests/test_gpu_parity.py). */
int dk_f32_libm_async(int fn, uint32_t first, uint32_t stride, uint64_t n, float* d_y, void* stream);
int dk_az_select_async(dk_ctx* ctx, float c, dk_az_state* d_eval, uint8_t* d_need_eval, void* stream);
int dk_az_backup_async(dk_ctx* ctx, const float* d_value, const float* d_logits, void* stream);
int dk_az_finish_async(dk_ctx* ctx, int temperature_mode, float temperature, uint32_t* d_visits, uint8_t* d_action,
                       void* stream);
/* IMPI autoregressive determinization: forward_pred_process_with_mask
 * (rs-doko-impi/src/forward.rs:392-661), the SamplingFn of ARSampling
 * (rs-doko-py-bridge/src/compare_impi/compare_impi.rs:84-105), batched over
 * n_info x samples lanes (lane = info * samples + sample, seed d_seeds[lane]).
 * Every guess of every lane is one row of a network batch, run by the caller:
 *   dk_ar_begin_async    lanes from the infostate records (dk_az_state: the packed
 *                        state plus its announcement list); *d_rounds = the largest
 *                        number of guesses of a lane (one network call each)
 *   repeat *d_rounds times:
 *     dk_ar_prepare_async  each running lane moves to its next guess (a card for
 *                          the next player with open slots, 12 x 3 steps; then the
 *                          hidden reservations) and writes its 311 encode_state_ipi
 *                          tokens to d_tokens[lane] (other rows keep their content:
 *                          start from a zeroed buffer); a lane with nothing left
 *                          to guess runs _is_consistent and its log draw
 *     (network: d_tokens [lanes][311] -> d_logits [lanes][33] f32)
 *     dk_ar_choose_async   mask, softmax(temperature), normalize, choose_weighted
 *   dk_ar_prepare_async  once more (finishes every lane)
 *   dk_ar_output_async   d_out[lane] = the sample (clone_with_different_hands_and_
 *                        reservations, state.rs:96-118) or the infostate itself;
 *                        d_status 0 Consistent, 1 NotConsistent (d_reason =
 *                        NotConsistentReason, is_consistent.rs:26-36), 2 where the
 *                        reference panics, 3 unfinished.
 * The infostate records must stay valid until dk_ar_output_async.
 * dk_ar_guesses_async: per infostate, the number of guesses (network calls) a lane of it
 * makes unless it stops early.  A lane with g guesses has a pending guess only in
 * rounds 0..g-1, so with the infostates ordered by descending g the rows of round r
 * are a prefix of the lanes and the network can run on that prefix alone (the
 * choose kernel reads d_logits only for lanes with a pending guess). */
int dk_ar_begin_async(dk_ctx* ctx, const dk_az_state* d_infostates, uint32_t n_info, uint32_t samples,
                      const uint64_t* d_seeds, float log_chance, uint32_t* d_rounds, void* stream);
int dk_ar_guesses_async(dk_ctx* ctx, const dk_az_state* d_infostates, uint32_t n_info, uint32_t* d_counts,
                        void* stream);
int dk_ar_prepare_async(dk_ctx* ctx, int32_t* d_tokens, void* stream);
int dk_ar_choose_async(dk_ctx* ctx, const float* d_logits, float temperature, void* stream);
int dk_ar_output_async(dk_ctx* ctx, dk_state* d_out, uint8_t* d_status, uint8_t* d_reason, void* stream);
/* The end of DefaultImpiPolicy::execute (compare_impi.rs:297-370) for AR samples:
 * d_successes[i] = consistent samples of infostate i (d_status == 0); an infostate with none
 * gets d_action[i] = FdoAllowedActions::random over its legal actions minus the five
 * announcements (SmallRng::seed_from_u64(d_seeds[i])); other entries of d_action are
 * left for the fusion to write. */
int dk_ar_fallback_async(dk_ctx* ctx, uint32_t n_info, uint32_t samples, const uint8_t* d_status, const uint64_t* d_allowed,
                         const uint64_t* d_seeds, uint8_t* d_action, uint32_t* d_successes, void* stream);

/* is_consistent (rs-full-doko/src/matching/is_consistent.rs:38-305): whether assumed hands
 * hands[4*i..] (reference bit layout) and assumed reservations reservations[4*i..] (FdoReservation,
 * DK_NONE = None; by player) are consistent with infostate record i, as the observer (its
 * current player) sees it.  reasons[i] = DK_NONE when consistent, else the NotConsistentReason
 * (is_consistent.rs:26-36: 0 HandSizeMismatch 1 NotInRemainingCards 2 RemainingCardsLeft
 * 3 AlreadyDiscardedColor 4 HasClubQueenButSomeoneElseAnnouncedWedding 5 HasNoClubQueenButAnnouncedRe
 * 6 HasClubQueenButAnnouncedKontra 7 WrongReservation 8 WrongReservationClubQ); 0xFE for a finished
 * infostate (the reference unwraps its current player). */
int dk_is_consistent_batch(dk_ctx* ctx, const dk_az_state* infostates, const uint64_t* hands, const uint8_t* reservations,
                           uint32_t n, uint8_t* reasons);

/* Game records for self-play.  dk_az_records_async: records of packed rs-full-doko states
 * without announcements (new games, DK_E_STATE otherwise).  dk_az_step_async:
 * take_action_by_action_index(action, skip_single = true) (full_doko.rs:121-157) on every
 * record whose action is not DK_NONE (a self-play move).  dk_az_encode_async: the network
 * input encode_state_pi (rs-doko-networks/src/full_doko/var1/encode_pi.rs:27-214),
 * tokens[n][311] int32. */
int dk_az_records_async(dk_ctx* ctx, const dk_state* d_states, uint32_t n, dk_az_state* d_out, void* stream);
int dk_az_step_async(dk_ctx* ctx, dk_az_state* d_records, const uint8_t* d_actions, uint32_t n, void* stream);
int dk_az_encode_async(dk_ctx* ctx, const dk_az_state* d_records, uint32_t n, int32_t* d_tokens, void* stream);

/* ---- AlphaZero network row kernels (bf16 activations [rows, d], d % 32 == 0, d <= 512) ----
 * The network itself (az_network.py) is PyTorch; these fuse its memory-bound row passes:
 * dk_net_embed_ln_bf16_async: x = sum of the six token embeddings of encode_state_pi
 *   (tables = 6 device pointers: object, position, player, subposition, team, phase; the sum in
 *   that order with bf16 rounding after each add, as torch), h = LayerNorm(x; gamma, beta, eps).
 * dk_net_add_ln_bf16_async: x += delta (delta may be NULL), h = LayerNorm(x).
 * `stream` is the caller's stream (torch's current stream). */
int dk_net_embed_ln_bf16_async(const int32_t* d_tokens, uint32_t batch, const void* const* tables, uint32_t d,
                               const void* gamma, const void* beta, float eps, void* x_out, void* h_out, void* stream);
int dk_net_add_ln_bf16_async(void* x_io, const void* delta, uint32_t rows, uint32_t d, const void* gamma, const void* beta,
                             float eps, void* h_out, void* stream);
/* dk_net_fc_gelu_bf16_async: y[rows][n] = GELU(x[rows][k] w[n][k]^T + bias[n]) with the exact
 * (erf) GELU of nn.GELU(): the first layer of a block's MLP (k = d = 160 or 256, n % 64 == 0),
 * bf16 in and out, f32 accumulation, the activation written once. */
int dk_net_fc_gelu_bf16_async(const void* x, const void* w, const void* bias, uint32_t rows, uint32_t k, uint32_t n,
                              void* y, void* stream);
/* dk_net_mlp_ln_bf16_async: the MLP half of a transformer block and the LayerNorm after it in
 * one pass (d = 160 with n_hidden % 64 == 0, or d = 256 with n_hidden % 32 == 0): delta = GELU(h w1^T + b1) w2^T + b2 (exact GELU; delta
 * rounded to bf16 as the unfused proj GEMM outputs it), x += delta (bf16), h_out = LayerNorm(x;
 * gamma, beta, eps).  w1 [n_hidden][d], w2 [d][n_hidden] (nn.Linear layout).  Replaces
 * dk_net_fc_gelu_bf16_async + the second GEMM + dk_net_add_ln_bf16_async of
 * TransformerBlock.py's MLP (az_doko.py:87-145). */
int dk_net_mlp_ln_bf16_async(const void* h, void* x_io, const void* w1, const void* b1, const void* w2, const void* b2,
                             uint32_t rows, uint32_t d, uint32_t n_hidden, const void* gamma, const void* beta, float eps,
                             void* h_out, void* stream);
/* dk_net_mlp_ln_f32x3_async: the same MLP half at the reference's precision (round 5): f32
 * activations and biases, bf16x3 products (each f32 operand split into bf16 hi + lo; three MFMAs
 * per k-step, ~16-bit product accuracy as hipBLASLt's f32 GEMMs at matmul precision "medium"
 * on gfx950).  w1_hi / w1_lo [n_hidden][d] and w2_hi / w2_lo [d][n_hidden] are the weights'
 * bf16 hi / lo parts, W2's columns in the split layout (az_network.mlp_split_bf16x3 makes all
 * four): d = 160, within every group of 16 hidden units units 4-7 and 8-11 swapped; d = 256,
 * within every group of 32 slot q holds unit 4 (q >> 3) + (q & 7) if (q & 7) < 4, else
 * 12 + 4 (q >> 3) + (q & 7);
 * x += (a W2^T + b2); h_out = LN(x).  d = 160 or 256, n_hidden % 32 == 0 (d = 256: % 64), n_hidden <= 1024.  Replaces F.linear + GELU + F.linear + add + LayerNorm of
 * rs-doko-py-bridge/python/az_doko.py:87-145 at f32. */
int dk_net_mlp_ln_f32x3_async(const float* h, float* x_io, const void* w1_hi, const void* w1_lo, const float* b1,
                              const void* w2_hi, const void* w2_lo, const float* b2, uint32_t rows, uint32_t d,
                              uint32_t n_hidden, const float* gamma, const float* beta, float eps, float* h_out,
                              void* stream);
/* dk_net_qkv_attn_ln_f32x3_async: the attention half at the reference's precision (round 5), one
 * workgroup per sample: Q, K, V = W h^T + b, softmax(K Q^T / sqrt(hd)), y = P V, x += y Wp^T + bp,
 * h_out = LN(x) -- f32 activations, bf16x3 products everywhere (operands split into bf16 hi + lo).
 * wqkv_hi / _lo [3d][d] (q | k | v rows, heads contiguous), wp_hi / _lo [d][d] the folded
 * out_proj / c_proj (Block.folded_proj), bp f32 [d].  d = 160 (4 heads of 40).  Replaces the qkv
 * F.linear, the attention core, the projection F.linear and add + LayerNorm of
 * rs-doko-py-bridge/python/az_doko.py:87-145 at f32. */
int dk_net_qkv_attn_ln_f32x3_async(const float* h, float* x_io, const void* wqkv_hi, const void* wqkv_lo, const float* bqkv,
                                   const void* wp_hi, const void* wp_lo, const float* bp, uint32_t batch, uint32_t heads,
                                   uint32_t head_dim, const float* gamma, const float* beta, float eps, float* h_out,
                                   void* stream);

/* dk_net_qkv_attn_ln_f32x3_ex_async / dk_net_mlp_ln_f32x3_ex_async (d = 256, 4 heads of 64; and
 * since round 6 d = 160, 4 heads of 40, x-input form only): the two halves above with the LayerNorm
 * moved into the consumer, so that a chain of halves moves the residual stream x only.  Input: h_in
 * [rows, d] as above, or h_in NULL and the kernel normalises x itself with (ln_in_gamma,
 * ln_in_beta, ln_in_eps) -- the LayerNorm the producer used to apply.  h_out NULL: only x is
 * updated (gamma / beta unused); otherwise h_out = LN(x) as above.
 * Row statistics (d = 160 only; NULL at d = 256): stats_out [rows][2] receives each new x row's
 * LayerNorm mean and 1 / sqrt(var + eps) (eps: the LayerNorm the next half applies); stats_in gives
 * the x-input form those statistics instead of reducing over the row (the d = 160 MLP half
 * requires them; the attention half computes them itself when stats_in is NULL).  stats_in and
 * stats_out may be the same buffer.  x_out (attention half only; NULL or x_io: in place): the new
 * x rows are written there and x_io is only read -- a branch that starts from a shared trunk's x
 * (the AlphaZero network's policy and value branches) without copying it first.  The same weights,
 * split layouts and validity rules (n_hidden % 64 == 0); DK_E_INVALID otherwise. */
int dk_net_qkv_attn_ln_f32x3_ex_async(const float* h_in, float* x_io, const float* ln_in_gamma, const float* ln_in_beta,
                                      float ln_in_eps, const void* wqkv_hi, const void* wqkv_lo, const float* bqkv,
                                      const void* wp_hi, const void* wp_lo, const float* bp, uint32_t batch, uint32_t heads,
                                      uint32_t head_dim, const float* gamma, const float* beta, float eps, float* h_out,
                                      const float* stats_in, float* stats_out, float* x_out, void* stream);
int dk_net_mlp_ln_f32x3_ex_async(const float* h_in, float* x_io, const float* ln_in_gamma, const float* ln_in_beta,
                                 float ln_in_eps, const void* w1_hi, const void* w1_lo, const float* b1, const void* w2_hi,
                                 const void* w2_lo, const float* b2, uint32_t rows, uint32_t d, uint32_t n_hidden,
                                 const float* gamma, const float* beta, float eps, float* h_out, const float* stats_in,
                                 float* stats_out, void* stream);
/* The heads at the reference's precision (round 5; PerClassAttentionMLPHead,
 * rs-doko-py-bridge/python/az_doko.py:28-56), f32 activations, bf16x3 MFMA products:
 * dk_net_class_pool_ln_f32_async: x [B, 62, d] -> out [C, B, d] (class-major) =
 *   LN(softmax(q_c x^T * scale) x) * ln_w[c] + ln_b[c]; queries / ln_w / ln_b [C, d] f32;
 *   C <= 64, d = 160 or 256.  The f32 form of dk_net_class_pool_ln_bf16_async.
 * dk_net_class_mlp_f32x3_async: pooled [C, B, d] -> out [B, C] = w2[c] . GELU(W1[c] a + b1[c])
 *   + b2[c] (exact erf GELU); w1_hi / w1_lo [C, d, d] bf16 (the split of W1), b1 / w2 [C, d],
 *   b2 [C] f32.  The class MLPs of the head's forward in one launch. */
int dk_net_class_pool_ln_f32_async(const float* x, uint32_t batch, uint32_t d, const float* queries, uint32_t classes,
                                   float scale, const float* ln_w, const float* ln_b, float eps, float* out, void* stream);
int dk_net_class_mlp_f32x3_async(const float* pooled, uint32_t batch, uint32_t d, uint32_t classes, const void* w1_hi,
                                 const void* w1_lo, const float* b1, const float* w2, const float* b2, float* out,
                                 void* stream);
/* dk_net_class_mlp_bf16_async: the bf16 network's class MLPs in one launch: pooled [C, B, d]
 * (dk_net_class_pool_ln_bf16_async's output) -> out [B, C] bf16 = w2[c] . GELU(W1[c] a + b1[c])
 * + b2[c] (f32 accumulation, exact erf GELU); w1 [C, d, d], b1 / w2 [C, d], b2 [C] bf16. */
int dk_net_class_mlp_bf16_async(const void* pooled, uint32_t batch, uint32_t d, uint32_t classes, const void* w1,
                                const void* b1, const void* w2, const void* b2, void* out, void* stream);
/* dk_net_class_pool_ln_bf16_async: PerClassAttentionMLPHead's attention pooling and each class
 * MLP's opening LayerNorm (az_doko.py:42-50): x [batch][62][d], queries [classes][d] (classes
 * <= 64), w = softmax(queries x^T * scale) over the 62 tokens, a = w x, out[c][b][:] =
 * LayerNorm(a[b][c]; ln_w[c], ln_b[c], eps), class-major [classes][batch][d].  d 160 or 256. */
int dk_net_class_pool_ln_bf16_async(const void* x, uint32_t batch, uint32_t d, const void* queries, uint32_t classes,
                                    float scale, const void* ln_w, const void* ln_b, float eps, void* out, void* stream);
/* dk_net_qkv_attn_ln_bf16_async: the whole attention half of a transformer block from
 * h = ln_1(x): qkv = h wqkv^T + bqkv (wqkv [3d][d], nn.MultiheadAttention.in_proj order q | k | v,
 * heads contiguous), then as dk_net_attn_ln_bf16_async.  h and h_out must not alias. */
int dk_net_qkv_attn_ln_bf16_async(const void* h, void* x_io, const void* wqkv, const void* bqkv, const void* wp, const void* bp,
                                  uint32_t batch, uint32_t heads, uint32_t head_dim, const void* gamma, const void* beta,
                                  float eps, void* h_out, void* stream);
/* dk_net_attn_ln_bf16_async: the attention half of a transformer block after its qkv projection,
 * in one pass per sample: y = attention core (as dk_net_attn62_bf16_async), delta = y wp^T + bp
 * (the folded out_proj / c_proj, wp [d][d]), x += delta (bf16), h_out = LayerNorm(x; gamma,
 * beta, eps).  heads = 4, head_dim 40 (d 160) or 64 (d 256). */
int dk_net_attn_ln_bf16_async(const void* qkv, void* x_io, const void* wp, const void* bp, uint32_t batch, uint32_t heads,
                              uint32_t head_dim, const void* gamma, const void* beta, float eps, void* h_out, void* stream);
/* dk_net_attn62_bf16_async: softmax(q k^T / sqrt(head_dim)) v for the networks' shape (62
 * tokens; heads x head_dim = 4 x 40 for the AlphaZero network, 4 x 64 for the IMPI network),
 * q/k/v read from the fused projection qkv[batch*62][3d] ([q | k | v], heads contiguous), the
 * heads' outputs written to y[batch*62][d]; bf16 MFMA, one wave per (sample, head). */
int dk_net_attn62_bf16_async(const void* qkv, void* y, uint32_t batch, uint32_t heads, uint32_t head_dim,
                             void* stream);

/* ---- f32 network row kernels: the networks at the reference's precision (f32 activations;
 * az_doko.py:379-400, 539-541).  d % 4 == 0, d <= 512; f32 tables / gamma / beta / activations.
 * dk_net_embed_ln_f32_async: x = e0[t0] + e1[t1] + ... + e5[t5] (f32, left to right), h = LN(x).
 * dk_net_add_ln_f32_async:   x += delta (delta may be NULL), h = LN(x).
 * dk_net_attn62_f32_async:   softmax(q k^T / sqrt(head_dim)) v on the f32 matrix cores (f32 products and sums),
 *                            62 tokens, q/k/v read from qkv[batch*62][3d]
 *                            (heads contiguous), y[batch*62][d]; head_dim 40 or 64.
 * dk_net_gelu_f32_async:     y = GELU(y) in place (exact erf form), n elements, n % 4 == 0. */
int dk_net_embed_ln_f32_async(const int32_t* d_tokens, uint32_t batch, const void* const* tables, uint32_t d,
                              const void* gamma, const void* beta, float eps, void* x_out, void* h_out, void* stream);
int dk_net_add_ln_f32_async(void* x_io, const void* delta, uint32_t rows, uint32_t d, const void* gamma, const void* beta,
                            float eps, void* h_out, void* stream);
int dk_net_attn62_f32_async(const void* qkv, void* y, uint32_t batch, uint32_t heads, uint32_t head_dim, void* stream);
int dk_net_gelu_f32_async(void* y, uint64_t n, void* stream);
/* The same with the producing GEMM's bias applied first (so the GEMM itself runs without its bias
 * epilogue: hipBLASLt's f32 GEMMs at matmul precision "medium" take ~2x longer with it,
 * profiles/r04/fp32_bias_probe.log).  bias may be NULL.
 * dk_net_add_bias_ln_f32_async: x += (delta + bias[col]), h = LN(x)   (torch: delta = F.linear(.., b))
 * dk_net_gelu_bias_f32_async:   y = GELU(y + bias[i % width]), width % 4 == 0, n % width == 0
 * dk_net_attn62_bias_f32_async: q, k, v = qkv + bqkv[3d] as they load, then as dk_net_attn62_f32_async */
int dk_net_add_bias_ln_f32_async(void* x_io, const void* delta, const void* bias, uint32_t rows, uint32_t d,
                                 const void* gamma, const void* beta, float eps, void* h_out, void* stream);
int dk_net_gelu_bias_f32_async(void* y, const void* bias, uint64_t n, uint32_t width, void* stream);
int dk_net_attn62_bias_f32_async(const void* qkv, const void* bqkv, void* y, uint32_t batch, uint32_t heads,
                                 uint32_t head_dim, void* stream);

/* ---- completion / errors / timing of *_async work -------------------------------
 * dk_sync: waits for the stream and returns the first device-side error
 * (DK_E_CAPACITY when a search ran out of child slots) since the last dk_sync, including
 * errors of search launches on that stream whose slot a later launch reused (more than
 * eight searches in flight without a dk_sync).
 * dk_last_search_ms: device time of the last search launch (HIP events recorded
 * on the launch stream around the kernel).
 */
int dk_sync(dk_ctx* ctx, void* stream);
int dk_last_search_ms(dk_ctx* ctx, float* ms);
/* Per-wave clocks of the last search launch's persistent grid (each workgroup stamps the
 * 100 MHz realtime counter when it starts and when the group queue has run dry for it):
 * out[0] = span first start -> last end (ms), out[1] = mean fraction of the span a wave had
 * work (1 - out[1] is the drain tail plus the launch ramp), out[2] = the first wave's end and
 * out[3] = the median wave's end (ms after the first start), out[4] = waves.  Measurement
 * only (the reference has no counterpart); waits for the launch. */
int dk_last_search_waves(dk_ctx* ctx, double* out);
/* The shader clock of the last search launch, from s_memtime / s_memrealtime stamps taken by
 * every wave at its start and end (measurement; no reference counterpart): out[0] = mean clock in
 * MHz (shader cycles / real time over all waves), out[1] / out[2] = the slowest / fastest wave's
 * clock, out[3] = mean shader cycles a wave was busy.  Makes a launch's time comparable across
 * boxes whose clocks differ (cycles per simulation). */
int dk_last_search_clocks(dk_ctx* ctx, double* out);
/* memory footprint of the node / state pools reserved by dk_create (bytes) */
uint64_t dk_pool_bytes(const dk_ctx* ctx);
/* Pool demand since dk_create (waits for `stream`): the most child slots one search used
 * (in either pool), the main pools' capacity per root, and how many roots overflowed it
 * and were searched again in the fallback pool. */
int dk_pool_high_water(dk_ctx* ctx, void* stream, uint32_t* slots, uint32_t* capacity, uint32_t* overflowed);

#ifdef __cplusplus
}
#endif
#endif /* DOKO_AMD_H */
