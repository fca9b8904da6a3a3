"""MI355X-native NRMS news-recommendation scoring (drop-in for
Maguire1999/NewsRecommendationSystem's ``model.NRMS``).

    from newsrecommendationsystem_amd import NRMS, NRMSConfig
"""
from .config import BaseConfig, NRMSConfig  # noqa: F401
from .nrms import NRMS  # noqa: F401

__all__ = ["NRMS", "NRMSConfig", "BaseConfig"]
