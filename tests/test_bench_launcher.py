"""bench.py's multi-GPU path on CPU: `--gpus 2` starts two ranks under
torch.distributed.run, each replays its own documents (config 2: weak scaling, gloo
barrier, max-over-ranks time) or its LPT share after rank 0's ingest (config 5:
all_to_all redistribution + digest gather to rank 0), and rank 0 prints one JSON line
with n_gpus 2.  At N=1 the line carries the digest parity check against the oracle.
Runs bench's code on the host emulation (tests/bench_emu_driver.py)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "bench_emu_driver.py")


def run(*args, timeout=300):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, DRIVER, *args], capture_output=True, text=True, timeout=timeout, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_launcher_config2_two_ranks():
    out = run("--gpus", "2", "--config", "config2", "--docs", "3", "--ops", "400", "--steps", "2", "--warmup", "1",
              "--no-cpu-baseline")
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    # every rank replays its own sample on the oracle; rank 0 reports the sum (N > 1 parity)
    assert out["parity"].startswith("SnapshotV1 digests == oracle on 6 docs (2 ranks"), out["parity"]
    assert out["value"] > 0 and out["steps"] == 2


def test_launcher_config5_two_ranks():
    out = run("--gpus", "2", "--config", "config5", "--docs", "5", "--steps", "1", "--warmup", "0",
              "--no-cpu-baseline")
    assert out["n_gpus"] == 2
    assert out["config"]["docs_total"] == 10
    assert out["parity"].startswith("status words clean on every rank")
    assert out["exchange"]["docs_checked"] == 10 and out["exchange"]["checksum_mismatch_docs"] == 0


def test_launcher_config5_two_ranks_oracle_parity():
    out = run("--gpus", "2", "--config", "config5", "--docs", "6", "--steps", "1", "--warmup", "0")
    assert out["n_gpus"] == 2 and out["config"]["docs_total"] == 12
    assert out["parity"].startswith("SnapshotV1 digests == oracle on 12 docs (2 ranks"), out["parity"]
    assert out["exchange"]["checksum_mismatch_docs"] == 0


def test_single_rank_digest_parity_against_oracle():
    out = run("--config", "config2", "--docs", "20", "--ops", "300", "--steps", "1", "--warmup", "0",
              "--cpu-seconds", "0.2")
    assert out["n_gpus"] == 1
    assert out["parity"].startswith("SnapshotV1 digests == oracle on"), out["parity"]
    assert out["cpu_baseline"]["kind"] == "port"
    assert out["roofline"]["bytes_pinned"].startswith("mt_doc_counters == oracle"), out["roofline"]


def test_config5_rank_shares_equal_one_rank_replay():
    """--shares 4: the four ranks' LPT shares of 20 documents replayed in turn give every
    document the SnapshotV1 digest a one-rank replay of all 20 gives (each share's rows are the
    send buffer's slice all_to_all_single would deliver)."""
    sh = run("--config", "config5", "--docs", "5", "--shares", "4", "--steps", "1", "--warmup", "0", "--no-cpu-baseline")
    one = run("--config", "config5", "--docs", "20", "--steps", "1", "--warmup", "0", "--no-cpu-baseline")
    assert len(sh["shares"]) == 4 and sum(x["docs"] for x in sh["shares"]) == 20
    assert all(x["status_clean"] for x in sh["shares"])
    assert sh["config"]["msgs_total"] == one["config"]["msgs_total"]
    assert sh["digest_xor"] == one["sharding"]["digest_xor"]
    assert sh["ms_per_step"] == max(x["ms_per_step"] for x in sh["shares"])
