"""Estimators and model persistence."""
from .multiclass import OneVsRestSVC
from .svc import SVC

__all__ = ["SVC", "OneVsRestSVC"]
