"""Alias module: Test.py imports ``from Runner_P128 import OptimizedQSC_P128`` (Test.py:6)."""
from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import QSC_P128 as OptimizedQSC_P128  # noqa: F401
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.runner import Y2HRunner  # noqa: F401
