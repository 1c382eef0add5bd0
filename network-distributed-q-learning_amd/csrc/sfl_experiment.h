// Timing-only experiment switches of the env kernels.  Each one removes or duplicates a piece of work
// to price it (the phase A/Bs of DESIGN.md §5); a library built with any of them computes WRONG results.
//
// They exist only as these constants.  A switch is set by its -D define (SFL_X_* / SFL_AB_*), and a
// define is accepted only together with SFL_EXPERIMENT, which build.py adds itself and which it refuses
// to combine with the product output path (libsfl.so).  The defines are part of the library's build id
// (build.py build_id), so an experiment library also fails the product loader's freshness check
// (_lib.Lib.check_fresh) unless the caller opts in (SFL_EXPERIMENTAL=1, bench.py --experimental), and
// bench.py then names the library and its defines in its JSON line.
#pragma once

#if !defined(SFL_EXPERIMENT) &&                                                                                \
    (defined(SFL_X_NOTICK) || defined(SFL_X_NOPF) || defined(SFL_X_NORNG) || defined(SFL_AB_NO_QST) ||         \
     defined(SFL_AB_NO_TOUCH) || defined(SFL_AB_NO_SLOT) || defined(SFL_AB_LOAD2) || defined(SFL_AB_STORE2) ||   \
     defined(SFL_X_NOSSQ) || defined(SFL_X_EPSCONST) || defined(SFL_AB_SLOT2) || defined(SFL_AB_QST2) ||         \
     defined(SFL_AB_TOUCH2))
#error "timing-only experiment switch without SFL_EXPERIMENT: build experiment libraries through build.py"
#endif

namespace sfl {
namespace xp {
#ifdef SFL_X_NOTICK
constexpr bool kNoTick = true;  // a tick only advances the clock (no train moves)
#else
constexpr bool kNoTick = false;
#endif
#ifdef SFL_X_NOPF
constexpr bool kNoPrefetch = true;  // the batch prefetch stages nothing
#else
constexpr bool kNoPrefetch = false;
#endif
#ifdef SFL_X_NORNG
constexpr bool kNoRng = true;  // no epsilon-greedy draws: every decision greedy
#else
constexpr bool kNoRng = false;
#endif
#ifdef SFL_AB_NO_QST
constexpr bool kNoQStore = true;  // the pending update's Q store is dropped
#else
constexpr bool kNoQStore = false;
#endif
#ifdef SFL_AB_NO_TOUCH
constexpr bool kNoTouch = true;  // key-set inserts dropped
#else
constexpr bool kNoTouch = false;
#endif
#ifdef SFL_AB_NO_SLOT
constexpr bool kNoSlot = true;  // (switch, train) slot stores dropped
#else
constexpr bool kNoSlot = false;
#endif
#ifdef SFL_AB_LOAD2
constexpr bool kLoadTwice = true;  // the launch's state load runs twice (its marginal cost)
#else
constexpr bool kLoadTwice = false;
#endif
#ifdef SFL_AB_STORE2
constexpr bool kStoreTwice = true;  // the launch's state store runs twice
#else
constexpr bool kStoreTwice = false;
#endif
#ifdef SFL_X_NOSSQ
constexpr bool kNoSeedSeqLoad = true;  // the SeedSequence-table value replaced by arithmetic on the index
#else
constexpr bool kNoSeedSeqLoad = false;
#endif
#ifdef SFL_X_EPSCONST
constexpr bool kEpsConst = true;  // epsilon = eps0 (no epsilon-table load)
#else
constexpr bool kEpsConst = false;
#endif
// Marginal cost of one write of the post step, with unchanged results: each write of the class issued a second
// time, to the same address, behind a compiler barrier (so that it is not merged away).  The round-4 verdict's
// slot write-back cache would remove one of a decision's two slot stores: SLOT2 bounds what that can gain.
#ifdef SFL_AB_SLOT2
constexpr bool kSlotTwice = true;  // every (switch, train) slot store of the fused post twice
#else
constexpr bool kSlotTwice = false;
#endif
#ifdef SFL_AB_QST2
constexpr bool kQStoreTwice = true;  // the pending update's Q store twice
#else
constexpr bool kQStoreTwice = false;
#endif
#ifdef SFL_AB_TOUCH2
constexpr bool kTouchTwice = true;  // the post's key-set inserts twice
#else
constexpr bool kTouchTwice = false;
#endif
}  // namespace xp
}  // namespace sfl
