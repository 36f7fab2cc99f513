from dgi.models.config import ModelConfig, PRESETS, get_config  # noqa: F401
