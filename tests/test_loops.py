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
