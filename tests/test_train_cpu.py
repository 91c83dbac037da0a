"""Host-side pieces of the training driver: config reading quirks
(scripts/train.py:110-119), directories, logger file formats and the
rolling metrics window (src/utils/logger.py)."""
import json

import numpy as np
import yaml

from training.trainer import DEFAULT_CONFIG, create_directories, load_config, ppo_config_from
from utils.logger import Logger, MetricsTracker, TensorBoardLogger


def test_ppo_config_reading_quirks(tmp_path):
    cfg = {"ppo": {"learning_rate": 1e-3}, "training": {"batch_size": 512, "num_epochs": 3}}
    c = ppo_config_from(cfg)
    assert c.learning_rate == 1e-3 and c.batch_size == 512
    assert c.num_epochs == 10  # training.num_epochs is ignored; ppo.num_epochs is read
    assert ppo_config_from({"ppo": {"num_epochs": 4}}).num_epochs == 4
    assert ppo_config_from({}).batch_size == 2048
    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump(DEFAULT_CONFIG))
    assert load_config(str(p)) == DEFAULT_CONFIG


def test_create_directories(tmp_path):
    cfg = {"paths": {"checkpoint_dir": str(tmp_path / "a"), "log_dir": str(tmp_path / "b")}}
    d = create_directories(cfg)
    assert d["checkpoint"].is_dir() and d["log"].is_dir() and str(d["results"]) == "results"
    assert d["results"].is_dir()
    d["results"].rmdir()


def test_logger_jsonl_and_summary(tmp_path):
    lg = Logger(str(tmp_path), "exp")
    lg.log({"fps": 10.0, "avg_score": np.float32(2.5), "n": np.int64(3)}, step=64)
    lg.log({"fps": 30.0, "avg_score": 4.5, "n": 5}, step=128)
    recs = [json.loads(x) for x in lg.log_file.read_text().splitlines()]
    assert [r["step"] for r in recs] == [64, 128] and recs[0]["avg_score"] == 2.5 and "timestamp" in recs[0]
    assert lg.get_mean("fps") == 20.0
    lg.save_summary()
    s = json.loads((tmp_path / "exp_summary.json").read_text())
    assert s["total_steps"] == 128 and s["metrics"]["fps"] == {"mean": 20.0, "std": 10.0, "min": 10.0,
                                                                "max": 30.0, "last": 30.0}
    off = Logger(str(tmp_path / "none"), "x", enabled=False)
    off.log({"a": 1.0})
    assert not (tmp_path / "none").exists()
    tb = TensorBoardLogger(str(tmp_path), "x", enabled=False)
    tb.log_metrics({"a": 1.0}, 1)
    tb.close()


def test_metrics_tracker_window():
    m = MetricsTracker(window_size=100)
    for v in range(250):
        m.add("s", v)
    assert m.get_mean("s") == np.mean(np.arange(150, 250)) and m.get_max("s") == 249 and m.get_min("s") == 150
    m.extend("t", range(5))
    assert m.get_last("t") == 4 and m.get_summary("t")["std"] == np.std(range(5))
    assert m.get_mean("missing") == 0.0
    m.reset()
    assert m.get_all_summaries() == {}
