"""§8f-3 template builders (host side) against the reference's data_prepare.get_prompts /
get_prompts_augmented / get_prompts_simple (data_prepare.py:287-537) on a synthetic
market_attribute.mat (the attribute submodule is absent offline), string for string."""
import numpy as np

from multimodal_reid_amd import synthetic as syn
from multimodal_reid_amd import templates
from conftest import golden


def test_template_builders_match_reference(tmp_path):
    g = golden("templates.npz")
    path = str(tmp_path / "attr.mat")
    syn.write_market_attribute_mat(path, n_ids=24, seed=5)
    ids, plain = templates.get_prompts(path)
    assert ids == list(g["ids"])
    assert [plain[i] for i in ids] == list(g["plain"])
    ids2, aug = templates.get_prompts_augmented(path)
    assert ids2 == ids
    for k, i in enumerate(ids):
        assert aug[i] == list(g["augmented"][k])
    _, simple = templates.get_prompts_simple(ids, 24)
    for k, i in enumerate(ids):
        assert simple[i] == list(g["simple"][k])
    assert len(aug[ids[0]]) == 56 and np.all([len(v) == 56 for v in aug.values()])
