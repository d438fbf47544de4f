"""Estimators and model persistence."""
from .svc import SVC

__all__ = ["SVC"]
