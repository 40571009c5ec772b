"""Multi-node launcher: reference hosts-file format -> one torchrun per node (dry run, no ssh)."""
from erasurehead_amd.launch import main, node_commands, read_hosts


def test_hosts_file_and_node_commands(tmp_path, capsys):
    hf = tmp_path / "hosts"
    hf.write_text("172.31.31.63\tdeeplearning-worker1\n# comment\n\n172.31.21.141 deeplearning-worker2\n10.0.0.3\n")
    hosts = read_hosts(str(hf))
    assert hosts == [("172.31.31.63", "deeplearning-worker1"), ("172.31.21.141", "deeplearning-worker2"),
                     ("10.0.0.3", "10.0.0.3")]
    cmds = node_commands(hosts, 8, "main.py", ["17", "1000", "10", "/d/"], port=29600, workdir="/repo")
    assert [c[0] for c in cmds] == ["172.31.31.63", "172.31.21.141", "10.0.0.3"]
    for j, (_, c) in enumerate(cmds):
        assert c.startswith("cd /repo && HSA_ENABLE_IPC_MODE_LEGACY=0 python -m torch.distributed.run")
        assert "--nnodes=3" in c and f"--node-rank={j}" in c and "--nproc-per-node=8" in c
        assert "--master-addr=172.31.31.63" in c and "--master-port=29600" in c
        assert c.endswith("main.py 17 1000 10 /d/")
    assert main(["--hosts", str(hf), "--gpus-per-node", "2", "--dry-run", "--", "9", "100"]) == 0
    out = capsys.readouterr().out.strip().splitlines()
    assert len(out) == 3 and out[1].startswith("172.31.21.141: ")
