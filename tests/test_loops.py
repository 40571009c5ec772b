"""The round-loop selection (engine/loops.py): one function, its table pinned, README generated from it."""
import os

import pytest

from erasurehead_amd.engine.loops import LoopInputs, loop_table, loop_table_markdown, select_round_loop

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _expected(t, delay, drain, instrument, checkpoint):
    """The table, written out independently of the function's code path."""
    if t == "gloo":
        return "python"
    if t == "local":
        if checkpoint or delay == "virtual":
            return "native pump"
        return "stream"
    if instrument or checkpoint or t != "ipc" or delay == "virtual":
        return "native pump"
    return "arbiter"


def test_every_combination_of_transport_delay_drain_instrument_checkpoint():
    rows = loop_table()
    assert len(rows) == 5 * 3 * 3 * 2 * 2
    for t, dl, dr, ins, ck, loop, why in rows:
        assert loop == _expected(t, dl, dr, ins, ck), (t, dl, dr, ins, ck, loop, why)
        assert why


def test_drain_never_changes_the_loop():
    by = {}
    for t, dl, dr, ins, ck, loop, _ in loop_table():
        by.setdefault((t, dl, ins, ck), set()).add(loop)
    assert all(len(v) == 1 for v in by.values())


@pytest.mark.parametrize("kw,loop", [
    (dict(world=8, transport="ipc", shared_gpu=True), "native pump"),
    (dict(world=8, transport="ipc", shared_gpu=True, device_master="on"), "arbiter"),
    (dict(world=8, transport="ipc", device_master="off"), "native pump"),
    (dict(world=8, transport="ipc", blocker="more than 64 worker ranks"), "native pump"),
    (dict(world=8, transport="ipc", resume=True), "native pump"),
    (dict(world=8, transport="ipc", verify_beta=True), "python"),
    (dict(world=1, native_loop=False), "python"),
    (dict(world=1, device_loop="graph"), "graph"),
    (dict(world=1, device_loop="off"), "native pump"),
    (dict(world=1, table_ondemand=True), "native pump"),
    (dict(world=8, transport="ipc", table_w64=True), "python"),
    (dict(world=1, gpu=False, transport="local"), "python"),
])
def test_overrides(kw, loop):
    got, why = select_round_loop(LoopInputs(**kw))
    assert got == loop, why


def test_readme_loop_table_is_generated():
    """README's "Round loops" table is loop_table_markdown() verbatim."""
    with open(os.path.join(ROOT, "README.md")) as f:
        text = f.read()
    assert loop_table_markdown() in text


@pytest.mark.parametrize("device_map,override,form", [
    (["0000:05:00.0"], "auto", "relaxed"),                                   # one rank
    (["0000:05:00.0"] * 8, "auto", "relaxed"),                               # 8 ranks time-share one GPU
    (["0000:05:00.0", "0000:15:00.0"], "auto", "strict"),                    # two GPUs: xGMI
    ([f"0000:{b:02x}:00.0" for b in (5, 0x15, 0x65, 0x75, 0x85, 0x95, 0xe5, 0xf5)], "auto", "strict"),  # a node
    (["a", "a", "b"], "auto", "strict"),                                     # any pair across devices
    (["0000:05:00.0", "0000:15:00.0"], "relaxed", "relaxed"),                # explicit opt-in only
    (["0000:05:00.0"] * 4, "strict", "strict"),
])
def test_release_form_from_device_map(device_map, override, form):
    """Round-5 verdict, first item: the strict release / acquire forms are the default whenever any two
    ranks sit on different GPUs; relaxed stays for ranks sharing one GPU (where it is measured) and is
    otherwise an explicit opt-in (ERASUREHEAD_RELEASE=relaxed)."""
    from erasurehead_amd.engine.loops import select_release_form

    got, why = select_release_form(device_map, override)
    assert got == form and why


def test_release_override_from_environment():
    from erasurehead_amd.engine.loops import release_override, select_release_form

    assert release_override({}) == "auto"
    assert release_override({"ERASUREHEAD_RELEASE": "Relaxed"}) == "relaxed"
    assert release_override({"ERASUREHEAD_RELEASE": " STRICT"}) == "strict"
    with pytest.raises(ValueError):
        select_release_form(["a", "b"], "fast")
