"""The GEMM dispatcher's tracked per-shape table (ops/gemm_table_mi355x.json; verdict r4 item 1c):
a shape in the table takes the table's pick with NO in-run timing (two boxes pick the same kernel),
a shape missing from it is timed; the table's picks are valid implementation ids, and the table
covers every GEMM kind / shape of the GPT-2 small and Llama-3 8B steps."""
import json

import pytest
import torch

from distributed_training_amd.ops import lm


def _fresh(monkeypatch, table_on=True):
    monkeypatch.setattr(lm, "_GEMM_CHOICE", {})
    monkeypatch.setattr(lm, "GEMM_PICK_SOURCE", {})
    monkeypatch.setattr(lm, "GEMM_TIMES", {})
    monkeypatch.setattr(lm, "_TABLE", {})
    monkeypatch.setattr(lm, "_TABLE_LOADED", [False])
    monkeypatch.setattr(lm, "_CACHE_LOADED", [True])
    monkeypatch.setattr(lm, "_gfx950", lambda: table_on)
    monkeypatch.delenv("DTA_GEMM", raising=False)
    monkeypatch.delenv("DTA_GEMM_TABLE", raising=False)
    monkeypatch.delenv("DTA_GEMM_CACHE", raising=False)


def test_table_is_valid_and_covers_the_lm_steps():
    doc = json.load(open(lm.TABLE_PATH))
    assert "gfx950" in doc["arch"] and doc["rounds"] >= 9
    base = lm.K64_TILES + lm.K64_TILES_KMAJOR
    valid = {0} | {lm.K64 + t for t in base} | {lm.K64 + (t | lm.SK_BIT) for t in lm._SK_TILES + lm._SK_TILES_KMAJOR}
    kinds = set()
    for key, e in doc["entries"].items():
        kind, dims = key.rsplit(" ", 1)
        M, N, K = (int(x) for x in dims.split("x"))
        assert M > 0 and N > 0 and K > 0
        assert e["pick"] in valid, key
        # the pick is the fastest median measured (hipBLASLt wins only when it is faster)
        us = e["us"]
        if kind not in ("fwd_gelu", "fwd_gelub"):  # (the GELU dual store keeps its 15 % handicap)
            assert us[e["pick_name"]] <= min(us.values()) * 1.0001, key
        if "in_step_pick" in e:  # an in-step override carries its evidence (same-box step A/B)
            assert e["in_step_pick"] in valid and e.get("in_step_evidence"), key
        kinds.add(kind)
    assert {"fwd", "fwdb", "dgrad", "wgrad", "head_fwd", "head_dgrad", "head_wgrad", "dgelu",
            "fwd_gelub"} <= kinds
    for key in ("fwd 8192x4096x4096", "dgrad 8192x14336x4096", "wgrad 28672x4096x8192", "head_fwd 8192x128256x4096",
                "fwdb 8192x2304x768", "head_fwd 8192x50304x768", "dgelu 8192x3072x768"):
        assert key in doc["entries"], key


def test_table_pick_needs_no_timing(monkeypatch):
    _fresh(monkeypatch)

    def boom(*a, **k):
        raise AssertionError("timed a shape that is in the tracked table")

    monkeypatch.setattr(lm, "_time_us", boom)
    table = lm.gemm_table()
    key = ("fwd", 8192, 4096, 4096)
    assert key in table
    cands = {0: lambda: None, **{lm.K64 + t: (lambda: None) for t in lm.K64_TILES}}
    c = lm._pick(*key, cands)
    assert c == table[key] and lm.GEMM_PICK_SOURCE[key] == "table"


def test_shape_missing_from_table_is_timed(monkeypatch):
    _fresh(monkeypatch)
    monkeypatch.setattr(lm, "_time_us", lambda cands, rounds=5, reps=4: {k: (10.0 if k else 12.0) for k in cands})
    cands = {0: lambda: None, lm.K64 + 5: lambda: None}
    c = lm._pick("fwd", 1024, 1024, 1024, cands)  # not a GPT-2 / Llama shape
    assert c == lm.K64 + 5 and lm.GEMM_PICK_SOURCE[("fwd", 1024, 1024, 1024)] == "timed"
    # library faster -> library
    monkeypatch.setattr(lm, "_time_us", lambda cands, rounds=5, reps=4: {k: (12.0 if k else 10.0) for k in cands})
    assert lm._pick("fwd", 2048, 1024, 1024, cands) == 0


def test_table_off_switch(monkeypatch):
    _fresh(monkeypatch)
    monkeypatch.setenv("DTA_GEMM_TABLE", "0")
    assert lm.gemm_table() == {}
    _fresh(monkeypatch, table_on=False)  # not a gfx950: no table
    assert lm.gemm_table() == {}


@pytest.mark.parametrize("mode", ["torch", "dta"])
def test_forced_modes_ignore_table(monkeypatch, mode):
    _fresh(monkeypatch)
    monkeypatch.setenv("DTA_GEMM", mode)
    if mode == "dta":
        monkeypatch.setattr(lm, "native", lambda: type("N", (), {"gemm64_tile": staticmethod(lambda M, N, K, t: 5)})())
    cands = {0: lambda: None, lm.K64 + 5: lambda: None}
    c = lm._pick("fwd", 8192, 4096, 4096, cands)
    assert c == (0 if mode == "torch" else lm.K64 + 5)
    assert torch.cuda.is_available() or True


def test_in_step_override_wins(monkeypatch, tmp_path):
    """An entry's documented ``in_step_pick`` (same-box step A/B) replaces its isolated-timing ``pick``."""
    _fresh(monkeypatch)
    doc = {"arch": "gfx950", "rounds": 15, "entries": {
        "dgrad 8192x768x3072": {"pick": lm.K64 + 7, "pick_name": "k64/t7", "us": {"k64/t7": 1.0},
                                "in_step_pick": lm.K64 + 6, "in_step_evidence": "test"},
        "fwd 64x64x64": {"pick": 0, "pick_name": "hipblaslt", "us": {"hipblaslt": 1.0}}}}
    p = tmp_path / "table.json"
    p.write_text(json.dumps(doc))
    monkeypatch.setattr(lm, "TABLE_PATH", str(p))
    table = lm.gemm_table()
    assert table[("dgrad", 8192, 768, 3072)] == lm.K64 + 6
    assert table[("fwd", 64, 64, 64)] == 0


def test_candidate_sets_respect_layouts_and_stream_k_rules():
    """The 192-wide tiles are offered for K-major operands only; stream-K forms only where the plain tile's
    last round leaves >= 10 % of the chip idle and the reduction is deep (K >= 8192), never for the TT layout;
    the stream-K plan keeps every tile within three workgroups (span >= ceil(nk / 2)) and covers all units."""
    from distributed_training_amd.ops import native

    C = native()
    names = lambda *a: {lm._impl_name(c) for c in lm.gemm_candidates(*a)}  # noqa: E731
    nt = names(8192, 2304, 768, False, False)
    assert {"k64/t11", "k64/t12"} <= nt and not any(n.endswith("sk") for n in nt)  # K = 768: no stream-K
    assert not ({"k64/t11", "k64/t12"} & names(8192, 2304, 768, False, True))
    deep = names(768, 3072, 8192, True, True)  # GPT-2 weight gradient: 36 tiles of 256 x 256
    assert "k64/t5sk" in deep and not any(n.startswith("k64/t11") or n.startswith("k64/t12") for n in deep)
    assert not any(n.endswith("sk") for n in names(768, 3072, 8192, True, False))  # TT: no stream-K
    assert not any(n.endswith("sk") for n in names(8192, 4096, 4096, False, False))  # 512 tiles: 2 full rounds
    for M, N, K, t in ((8192, 768, 3072, 6), (6144, 4096, 8192, 5), (8192, 768, 50304 // 64 * 64, 5), (256, 384, 448, 12)):
        tiles, grid, span = C.gemm64_sk_plan(M, N, K, t | lm.SK_BIT)
        nk = K // 64
        assert tiles > 0 and span >= (nk + 1) // 2 and grid * span >= tiles * nk > (grid - 1) * span, (M, N, K, t)
    assert C.gemm64_sk_plan(8192, 768, 3072, 3 | lm.SK_BIT)[0] == 0  # four-phase / non-stream-K base tile


def test_big_operands_leave_out_descriptor_only_tiles():
    """An operand spanning >= 2 GiB (GPT-2 at B = 32: the [32768, 50304] logit gradient) takes no candidate that
    DMAs only through 32-bit buffer descriptors (192-wide, stream-K, W4): they would refuse the launch."""
    base = {lm._impl_name(c) for c in lm.gemm_candidates(32768, 768, 50304, False, True)}
    big = {lm._impl_name(c) for c in lm.gemm_candidates(32768, 768, 50304, False, True, big=True)}
    assert any(n.endswith("sk") for n in base) and "k64/t10" in base
    assert big and not any(n.endswith("sk") or n in ("k64/t10", "k64/t11", "k64/t12") for n in big)
    x = torch.empty(0, dtype=torch.bfloat16)
    assert not lm._big(x) and lm._big(torch.empty(32768, 50304, dtype=torch.bfloat16, device="meta"))
    assert not lm._big(torch.empty(8192, 50304, dtype=torch.bfloat16, device="meta"))
