"""Config layering: defaults < YAML file < DML_* env < CLI / overrides."""
import argparse

import pytest

from cs230_distributed_machine_learning_amd.config import Config


def test_yaml_env_cli_layering(tmp_path, monkeypatch):
    f = tmp_path / "dml.yaml"
    f.write_text("port: 6001\nchunk_target_s: 0.5\nkeep-models: all\ndp_auto_gb: '12'\n"
                 "algo_weight: {RandomForestClassifier: 2}\n")
    monkeypatch.delenv("DML_CONFIG", raising=False)
    cfg = Config.from_env(config_file=str(f))
    assert (cfg.port, cfg.chunk_target_s, cfg.keep_models, cfg.dp_auto_gb) == (6001, 0.5, "all", 12.0)
    assert cfg.algo_weight == {"randomforestclassifier": 2.0}
    monkeypatch.setenv("DML_PORT", "7001")
    monkeypatch.setenv("DML_CONFIG", str(f))
    cfg = Config.from_env()
    assert cfg.port == 7001 and cfg.chunk_target_s == 0.5          # env beats the file
    ap = argparse.ArgumentParser()
    Config.add_cli(ap)
    cfg = Config.from_args(ap.parse_args(["--port", "8001", "--dp-min-cells", "10"]))
    assert cfg.port == 8001 and cfg.dp_min_cells == 10 and cfg.keep_models == "all"   # CLI beats env


def test_unknown_config_key_rejected(tmp_path, monkeypatch):
    monkeypatch.delenv("DML_CONFIG", raising=False)
    f = tmp_path / "bad.yaml"
    f.write_text("prot: 1\n")
    with pytest.raises(ValueError, match="prot"):
        Config.from_env(config_file=str(f))
