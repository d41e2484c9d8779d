"""Compatibility entry point: ``python Runner_P128_QuantumNAT_onchipQNN.py`` trains the quantum
scenario classifier and reports the wall time, as the reference's __main__ does; ``Y2HRunner``
keeps the reference's attributes and methods (see train/runner.py)."""
import sys
import time

from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.runner import Y2HRunner  # noqa: F401

if __name__ == "__main__":
    runner = Y2HRunner()
    print("=== Training Quantum Scenario Classifier ===")
    t0 = time.time()
    runner.train_QSC_P128()
    print(f"Quantum Scenario Classifier training time: {(time.time() - t0) / 60:.2f} minutes")
    print("HDCE and QML training completed!")
    sys.exit(0)
