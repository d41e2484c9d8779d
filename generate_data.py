"""The ``generate_data`` module the reference imports but does not ship (R:16, T:7):
``DatasetFolder_DML``, ``DatasetFolder``, ``generate_datapair`` and ``generate_MMSE_estimate``,
backed by the synthetic DeepMIMO-shaped generator of this framework."""
from quantum_distributed_machine_learning_ris_channel_estimation_amd.data.baselines import generate_MMSE_estimate  # noqa: F401
from quantum_distributed_machine_learning_ris_channel_estimation_amd.data.datasets import (  # noqa: F401
    DatasetFolder, DatasetFolder_DML, generate_datapair)
