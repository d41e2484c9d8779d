"""Compatibility entry point: ``python Test.py`` runs the NMSE-vs-SNR / scenario-accuracy sweep
(reference Test.py __main__) with ``model_val`` from train/evaluate.py."""
import sys

from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.evaluate import model_val  # noqa: F401

if __name__ == "__main__":
    test = model_val()
    print(f"Using device: {test.device}")
    print("Starting HDCE with Quantum vs Classical comparison test...")
    test.indicator = -1
    sys.exit(test.test_for_CE_P128_for_all_scenarios())
