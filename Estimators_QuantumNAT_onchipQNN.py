"""Compatibility entry point for ``from Estimators_QuantumNAT_onchipQNN import ...``.

The reference module (Estimators_QuantumNAT_onchipQNN.py) defines the estimator classes on
top of PennyLane; here they are the MI355X-native implementations of
quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators (same class
names, constructor arguments and state_dict keys; the VQC runs on HIP / C++ simulators).
"""
from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import (  # noqa: F401
    DCE_P128, FC_P128, NMSE_cuda, NMSELoss, QSC_P128, SC_P128, Conv_P128, QuantumLayer)

# The reference sets this from ``import pennylane``; the native simulator needs no PennyLane.
PENNYLANE_AVAILABLE = False
NATIVE_QUANTUM_BACKEND = True
