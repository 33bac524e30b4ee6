"""kyverno_amd — MI355X-native batch engine for Kyverno's validate.pattern hot path.

Public surface:
  kyverno_amd.batch   PolicySet / Batch / validate()  (batch engine.Validate over the C ABI)
  kyverno_amd.engine  PolicyContext / validate()      (per-call engine.Validate mirror)
  kyverno_amd.cli     `python -m kyverno_amd apply ...` (kyverno apply mirror)
"""
__version__ = "0.1.0"
