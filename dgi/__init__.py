"""dgi — MI355X-native distributed GPU inference runtime.

Layers:
  dgi.csrc      hand-written CDNA4 HIP kernels + torch op bindings (gfx950)
  dgi.ops       kernel entry points (HIP on GPU, torch references on CPU)
  dgi.models    Llama-3 configs and the native decoder
  dgi.kv        paged block pool, radix prefix cache, pinned-host CPU tier
  dgi.sched     iteration-level continuous-batching scheduler
  dgi.runtime   model runner, hipGraph decode capture
  dgi.parallel  RCCL fabric, layer pipeline, prefill/decode disaggregation
  dgi.spec      EAGLE-3 style speculative decoding
  dgi.engine    LLMEngine (single device or one pipeline stage)
"""
__version__ = "0.1.0"
