"""Model-config loading (utils.load_config, utils.py:26-59) and target-instrument selection
(utils.prefer_target_instrument, utils.py:480-499)."""
import yaml


class ConfigDict(dict):
    """Attribute-access dict standing in for ml_collections.ConfigDict (the reference's config
    type): ``cfg.audio.chunk_size``, ``'normalize' in cfg.inference``, ``getattr(cfg.training,
    'use_amp', True)`` all behave as with ConfigDict."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = wrap(v)

    def to_dict(self):
        return {k: (v.to_dict() if isinstance(v, ConfigDict) else v) for k, v in self.items()}


def wrap(o):
    if isinstance(o, ConfigDict):
        return o
    if isinstance(o, dict):
        return ConfigDict({k: wrap(v) for k, v in o.items()})
    if isinstance(o, list):
        return [wrap(v) for v in o]
    return o


class _Loader(yaml.SafeLoader):
    """SafeLoader + the !!python/tuple tag that released configs use (helpers.py:81-86)."""


_Loader.add_constructor("tag:yaml.org,2002:python/tuple", lambda ld, node: tuple(ld.construct_sequence(node)))


def load_config(model_type: str, config_path: str):
    """utils.load_config: YAML -> ConfigDict (no arbitrary-object construction)."""
    try:
        with open(config_path, "r") as f:
            return wrap(yaml.load(f, Loader=_Loader))
    except FileNotFoundError:
        raise FileNotFoundError(f"Configuration file not found at {config_path}")
    except Exception as e:
        raise ValueError(f"Error loading configuration: {e}")


def prefer_target_instrument(config):
    t = getattr(config.training, "target_instrument", None)
    if t:
        return [t]
    return list(config.training.instruments)
