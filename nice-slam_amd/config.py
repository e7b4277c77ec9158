"""YAML config loading with `inherit_from` and recursive merge (src/config.py:10-59)."""
from __future__ import annotations

import yaml


def update_recursive(dict1, dict2):
    """Merge dict2 into dict1 (nested dicts merged, leaves overwritten)."""
    for k, v in dict2.items():
        if k not in dict1:
            dict1[k] = dict()
        if isinstance(v, dict):
            update_recursive(dict1[k], v)
        else:
            dict1[k] = v


def load_config(path, default_path=None):
    """Load `path`, resolving `inherit_from` chains, then defaults from `default_path`."""
    with open(path, "r") as f:
        cfg_special = yaml.safe_load(f)
    inherit_from = cfg_special.get("inherit_from")
    if inherit_from is not None:
        cfg = load_config(inherit_from, default_path)
    elif default_path is not None:
        with open(default_path, "r") as f:
            cfg = yaml.safe_load(f)
    else:
        cfg = dict()
    update_recursive(cfg, cfg_special)
    return cfg
