"""ForestTiers: DML_TIER_<FIELD> overrides reach every field, feature-group sizes stay clamped
to the LDS budget, and regression builds get their own large-tier chunk (ops/forest_ops.py)."""
from cs230_distributed_machine_learning_amd.ops.forest_ops import ForestTiers


def test_env_overrides_reach_feature_group_fields(monkeypatch):
    monkeypatch.setenv("DML_TIER_KG_LARGE", "8")
    monkeypatch.setenv("DML_TIER_KG_BLOCK", "12")
    monkeypatch.setenv("DML_TIER_KG_LARGE_REG", "6")
    monkeypatch.setenv("DML_TIER_CHUNK_REG", "8192")
    t = ForestTiers().fitted(3)
    assert (t.kg_large, t.kg_block, t.kg_large_reg, t.chunk_reg) == (8, 12, 6, 8192)


def test_feature_groups_clamped_to_lds_budget(monkeypatch):
    monkeypatch.setenv("DML_TIER_KG_LARGE", "64")
    t = ForestTiers().fitted(101)            # 101 channels x 256 bins x 4 B = ~101 KB per feature
    assert t.kg_large == 1 and t.kg_block == 1 and t.kg_wave == 1
    t = ForestTiers().fitted(4)              # regression: 4 KB per feature
    assert t.kg_large == 24 and t.kg_large_reg == 16 and t.kg_wave == 4


def test_regression_defaults():
    t = ForestTiers().fitted(4)
    assert t.chunk_reg == 4096 and t.chunk == 16384


def test_forest_tiers_binary_wave_max(monkeypatch):
    """Binary classification (3 histogram channels) caps the wave tier at wave_max_bin; other
    builds keep wave_max; DML_TIER_WAVE_MAX overrides both (ops/forest_ops.py ForestTiers.fitted)."""
    from cs230_distributed_machine_learning_amd.ops.forest_ops import ForestTiers

    monkeypatch.delenv("DML_TIER_WAVE_MAX", raising=False)
    t = ForestTiers()
    assert t.fitted(3).wave_max == t.wave_max_bin == 256
    assert t.fitted(4).wave_max == t.wave_max == 512      # regression / 3 classes
    assert t.fitted(6).wave_max == 512
    monkeypatch.setenv("DML_TIER_WAVE_MAX", "384")
    assert t.fitted(3).wave_max == 384 and t.fitted(4).wave_max == 384
