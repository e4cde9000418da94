"""MI355X drop-in for the reference's ``optimizer`` package
(synthetic_static_obs/optimizer/).  ``from optimizer import cem`` then
``cem.CEM(...)`` exactly as ``S/main_mpc.py:5-6,82-83`` does."""
