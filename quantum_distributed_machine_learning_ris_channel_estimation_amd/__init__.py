"""MI355X-native hybrid quantum-classical RIS channel-estimation framework.

Capabilities of Fazilaton-Nisha/Quantum-Distributed-Machine-Learning-RIS-Channel-Estimation
(HDCE estimator, classical + variational-quantum scenario classifiers, LS/MMSE baselines,
NMSE-vs-SNR evaluation), re-designed for AMD Instinct MI355X (gfx950): hand-written HIP
kernels, HBM-resident data, fused 9-stream steps, HIP graphs, RCCL data parallelism.
"""
__version__ = "0.1.0"

from .config import EvalConfig, RunnerConfig  # noqa: F401
