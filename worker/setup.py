"""pip-installable worker package (reference worker/setup.py).

The HIP kernels live in the ``dgi`` package at the repository root and are
built in-tree (``python -c 'from dgi.build import build; build()'``);
this setup only installs the worker daemon.
"""
from setuptools import find_packages, setup

setup(
    name="gpu-worker",
    version="1.0.0",
    description="Distributed GPU inference worker (AMD Instinct MI355X)",
    python_requires=">=3.9",
    packages=find_packages(),
    py_modules=["api_client", "batch_processor", "cli", "config", "direct_server", "machine_id", "main"],
    install_requires=["torch>=2.4", "httpx>=0.25", "pyyaml>=6.0", "pydantic>=2.0", "fastapi>=0.100",
                      "uvicorn>=0.23"],
    extras_require={"hf": ["transformers>=4.40", "safetensors"], "image": ["diffusers>=0.24"],
                    "grpc": ["grpcio>=1.60", "protobuf>=4"]},
    entry_points={"console_scripts": ["gpu-worker=cli:main"]},
)
