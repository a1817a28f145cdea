"""handel_amd — MI355X-native BN256 BLS verification engine for Handel.

The product path is the HIP library handel_amd/_build/libhandel_gpu.so
(sources in handel_amd/csrc, C ABI in include/handel_gpu.h). This package is
the Python host side: `engine.Engine` (one GPU context), `bn256` (a mirror of
the reference's bn256/go plugin API), `processing` / `sigprocessing` (the
batched replacement for processing.go's one-at-a-time evaluator), `service`
(one GPU-owning verifier process serving many client processes) and the
host-side data formats (`partitioner`, `packets`, `registry`).
"""

__all__ = ["engine", "bn256", "processing", "sigprocessing", "partitioner", "packets", "registry", "service",
           "distributed"]
