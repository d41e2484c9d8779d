"""Alias module: Test.py imports the estimators as ``from Estimators import ...`` (Test.py:5)."""
from Estimators_QuantumNAT_onchipQNN import *  # noqa: F401,F403
from Estimators_QuantumNAT_onchipQNN import DCE_P128, FC_P128, NMSE_cuda, NMSELoss, QSC_P128, SC_P128, Conv_P128  # noqa: F401
