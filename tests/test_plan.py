"""Host-side enumeration of the k_step dispatch plan (no GPU needed).

gpf_plan_check (include/gpfit.h) builds the launch list run_factor issues (num_groups,
split_k, step_group and the grid sizing in csrc/gpfit_api.hip) and decodes every
workgroup of every launch with the kernel's own decoder (gpf::step_decode). Every
(block column, particle, tile) must be computed exactly once: one whole-tile workgroup, or
all S depth pieces exactly once (the flat finish's counters of that tile);
pieces must stay inside the split-K buffers and concurrent particle groups must not share
partial slots or counters. This is the structural guard for races like the v14 duplicate of
the last block column's w = 0 tile.
"""
import os

import pytest

import gpfit

NT = list(range(1, 21)) + [31, 32, 33, 64, 127, 128, 129, 130]

ENVS = [
    {},                                            # the defaults (persistent where slot-bound)
    {"GPF_PERSIST": "1"},                          # the persistent factorisation everywhere (nt >= 3)
    {"GPF_GROUPS": "2"}, {"GPF_GROUPS": "3"}, {"GPF_GROUPS": "4"},
    {"GPF_SPLIT_K": "2"}, {"GPF_SPLIT_K": "7"}, {"GPF_SPLIT_K": "16"},
    {"GPF_SPLIT_K": "7", "GPF_GROUPS": "3"},
    {"GPF_STEP_GROUP": "1"}, {"GPF_STEP_GROUP": "2", "GPF_GROUPS": "2"},
    {"GPF_EARLY_DIAG": "1"}, {"GPF_EARLY_DIAG": "0"},
    {"GPF_EARLY_DIAG": "1", "GPF_GROUPS": "3"},
    {"GPF_DEFER_SYRK": "0"}, {"GPF_DEFER_SYRK": "0", "GPF_EARLY_DIAG": "1"},
    {"GPF_DEFER_SYRK": "0", "GPF_EARLY_DIAG": "1", "GPF_GROUPS": "2"},
    {"GPF_SPLIT_K_SLOTS": "512"}, {"GPF_SPLIT_K_SLOTS": "64", "GPF_SPLIT_K_MINCH": "1"},
    {"GPF_SPLIT_K": "3", "GPF_SPLIT_K_SLOTS": "1000", "GPF_SPLIT_K_MINCH": "1", "GPF_GROUPS": "2"},
    {"GPF_REORDER": "0"}, {"GPF_REORDER": "0", "GPF_EARLY_DIAG": "1"},  # r4: the reordered dispatch off
    {"GPF_EARLY_DIAG": "1", "GPF_GROUPS": "2"},                         # reordered where it fits, two groups
    {"GPF_PAIR": "1"}, {"GPF_PAIR": "1", "GPF_GROUPS": "1"},            # r6: paired block columns
    {"GPF_PAIR": "1", "GPF_GROUPS": "3"}, {"GPF_PAIR": "1", "GPF_EARLY_DIAG": "0", "GPF_GROUPS": "1"},
    {"GPF_LA_ALL": "1"}, {"GPF_LA_ALL": "1", "GPF_EARLY_DIAG": "1", "GPF_GROUPS": "2"},  # r6: look-ahead pieces
    {"GPF_LA_ALL": "0"}, {"GPF_LA_ALL": "1", "GPF_LA_ALL_PB": "2", "GPF_LA_ALL_FIRST": "0"},
    {"GPF_LA_ALL": "1", "GPF_LA_ALL_PB": "3", "GPF_EARLY_DIAG": "1", "GPF_LA_ALL_FROM": "1"},
    {"GPF_LA_ALL": "1", "GPF_LA_ALL_FROM": "3"}, {"GPF_LA_ALL": "1", "GPF_LA_ALL_FROM": "-3"},
]


@pytest.fixture
def env(monkeypatch):
    def apply(kv):
        for k in ("GPF_GROUPS", "GPF_SPLIT_K", "GPF_STEP_GROUP", "GPF_EARLY_DIAG",
                  "GPF_DEFER_SYRK", "GPF_SPLIT_K_SLOTS", "GPF_SPLIT_K_MINCH", "GPF_PERSIST", "GPF_REORDER",
                  "GPF_PAIR", "GPF_LA_ALL", "GPF_LA_ALL_PB", "GPF_LA_ALL_FIRST", "GPF_LA_ALL_FROM"):
            monkeypatch.delenv(k, raising=False)
        if kv and "GPF_PERSIST" not in kv:  # the launch-plan knobs: on the per-block-column launches
            monkeypatch.setenv("GPF_PERSIST", "0")
        for k, v in kv.items():
            monkeypatch.setenv(k, v)
    return apply


@pytest.mark.parametrize("kv", ENVS, ids=lambda kv: ",".join(f"{k}={v}" for k, v in kv.items()) or "default")
def test_every_tile_has_exactly_one_finisher(env, kv):
    env(kv)
    seen_split = seen_groups = seen_persist = seen_pairs = 0
    for nt in NT:
        # all chunk sizes up to 64 at small nt; a spread at large nt (the check is O(pc nt^2))
        pcs = range(1, 65) if nt <= 33 else (1, 2, 7, 8, 15, 16, 17, 31, 32, 33, 63, 64)
        for pc in pcs:
            st = gpfit.plan_check(pc, nt)
            if st["persistent"]:  # one launch, every tile an item, one SYRK item per column 1 .. nt-2
                assert (st["launches"], st["groups"], st["split_tiles"], st["diag_workgroups"]) == (1, 1, 0, 0)
                assert st["whole_tiles"] == pc * (nt - 1) * nt and st["syrk_workgroups"] == pc * max(0, nt - 2)
                assert st["workgroups"] == st["whole_tiles"] + st["syrk_workgroups"]
                seen_persist += 1
                continue
            assert st["launches"] == (nt * st["groups"] if nt > 1 else 0)
            assert st["whole_tiles"] + st["split_tiles"] == pc * (nt - 1) * nt  # every (J, p, w)
            # early diagonal factor: one diagonal workgroup per particle in every launch
            assert st["diag_workgroups"] in (0, pc * nt if nt > 1 else 0)
            # deferred diagonal update: one SYRK workgroup per particle in launches 1 .. nt-2,
            # except under the all-tile split (which keeps the per-tile look-ahead)
            # (paired block columns: only the lead launches carry them; the follow launch's critical
            # tile finishes the diagonal block the lead's partial SYRK started)
            # (the C-side check counts them per launch: one per particle in every lead launch, none in a
            # follow launch; groups whose size is not a multiple of 8 stay unpaired)
            assert st["syrk_workgroups"] in (0, pc * max(0, nt - 2)) or st["lead_launches"] > 0
            assert st["syrk_workgroups"] == 0 or st["S"] == 1
            seen_split += st["split_tiles"] > 0
            seen_groups += st["groups"] > 1
            seen_pairs += st["lead_launches"] > 0
            if st["lead_launches"]:  # leads at odd J <= nt-2 in every paired group
                assert st["lead_launches"] % ((nt - 1) // 2) == 0 and st["lead_launches"] <= st["groups"] * ((nt - 1) // 2)
    if kv.get("GPF_SPLIT_K") or not kv:
        assert seen_split, "the sweep never reached a split launch"
    if kv.get("GPF_GROUPS", "1") != "1":
        assert seen_groups, "the sweep never reached a multi-group plan"
    if not kv or kv.get("GPF_PERSIST") == "1":
        assert seen_persist, "the sweep never reached the persistent factorisation"
    if kv.get("GPF_PAIR") == "1" and kv.get("GPF_EARLY_DIAG") != "1":
        assert seen_pairs, "the sweep never reached a paired plan"


def test_default_plans_of_the_baseline_configs(env):
    """The schedules the bench and the GPU tests rely on."""
    env({})
    # configs C and D: per-block-column launches on two concurrent group streams; config E's
    # share (128 block columns): the persistent factorisation, one launch of 128 x 127 tiles + 126
    # SYRK items per particle
    c = gpfit.plan_check(64, 32)            # config C
    assert (c["persistent"], c["groups"], c["Smax"]) == (0, 2, 1)
    d = gpfit.plan_check(32, 32)            # config D's per-GPU share
    assert (d["persistent"], d["groups"]) == (0, 2)
    e = gpfit.plan_check(16, 128)           # config E's per-GPU share at N=16384
    assert (e["persistent"], e["launches"], e["groups"]) == (1, 1, 1)
    assert e["workgroups"] == 16 * (128 * 127 + 126)
    env({"GPF_PERSIST": "1"})               # ... C persistent on request: 64 x (32 x 31 + 30) items
    assert gpfit.plan_check(64, 32)["workgroups"] == 64 * (32 * 31 + 30)
    env({"GPF_PERSIST": "0"})               # ... E on the launches: two concurrent groups
    e0 = gpfit.plan_check(16, 128)
    assert (e0["groups"], e0["diag_workgroups"], e0["syrk_workgroups"]) == (2, 0, 16 * 126)
    env({})
    b = gpfit.plan_check(32, 8)             # config B: one group, no split
    assert b["groups"] == 1 and b["S"] == 1 and b["Smax"] == 1 and b["split_tiles"] == 0
    env({})
    one = gpfit.plan_check(1, 32)           # prediction: single particle, all tiles split
    # every tile in at least SPLIT_MINP (4) pieces, J = 0's zero-depth tiles included (the flat
    # finish spreads their triangular multiply and diagonal update over the pieces' CUs)
    assert one["S"] > 1 and one["whole_tiles"] == 0
    # balanced pieces: every launch fits one workgroup per CU (255 + the diagonal workgroup),
    # and the critical tile of the deep launches gets the most pieces
    assert one["workgroups"] <= 32 * 256 and one["Smax"] > 8
    # early diagonal factor where launches leave slots idle (B, the prediction), the fused factor
    # in the persistent factorisation (C, D's and E's shares)
    assert (c["diag_workgroups"], d["diag_workgroups"], e["diag_workgroups"]) == (0, 0, 0)
    assert b["diag_workgroups"] == 32 * 8 and one["diag_workgroups"] == 32
    # deferred diagonal update (one SYRK workgroup / item per particle and column 1 .. nt-2)
    # everywhere but the all-tile split of the prediction
    assert (b["syrk_workgroups"], c["syrk_workgroups"]) == (32 * 6, 64 * 30)
    assert (d["syrk_workgroups"], e["syrk_workgroups"], one["syrk_workgroups"]) == (32 * 30, 16 * 126, 0)


def test_early_diag_override(env):
    env({"GPF_EARLY_DIAG": "1", "GPF_PERSIST": "0"})
    assert gpfit.plan_check(64, 32)["diag_workgroups"] == 64 * 32
    env({"GPF_EARLY_DIAG": "0"})
    assert gpfit.plan_check(32, 8)["diag_workgroups"] == 0


def test_defer_syrk_override(env):
    env({"GPF_DEFER_SYRK": "0", "GPF_PERSIST": "0"})
    assert gpfit.plan_check(32, 8)["syrk_workgroups"] == 0
    assert gpfit.plan_check(64, 32)["syrk_workgroups"] == 0
    env({"GPF_DEFER_SYRK": "1", "GPF_SPLIT_K": "4"})  # the all-tile split never defers
    assert gpfit.plan_check(8, 16)["syrk_workgroups"] == 0


def test_persistent_override(env):
    env({"GPF_PERSIST": "0"})
    assert gpfit.plan_check(64, 32)["persistent"] == 0
    env({"GPF_PERSIST": "1"})
    assert gpfit.plan_check(4, 8)["persistent"] == 1 and gpfit.plan_check(4, 2)["persistent"] == 0  # (nt >= 3)
    assert gpfit.plan_check(1, 32)["persistent"] == 0  # the prediction's single particle keeps its split launches


def test_env_is_read_per_call(env):
    env({"GPF_GROUPS": "4"})
    assert gpfit.plan_check(32, 32)["groups"] == 4
    env({"GPF_GROUPS": "1"})
    assert gpfit.plan_check(32, 32)["groups"] == 1
    assert os.environ.get("GPF_GROUPS") == "1"
