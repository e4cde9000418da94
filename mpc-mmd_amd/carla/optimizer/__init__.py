"""Drop-in replacement of the reference's CARLA optimizer package
(``carla/optimizer/``): ``from optimizer import cem`` with this directory's
parent (``mpc-mmd_amd/carla``) on ``sys.path``, as ``carla/main_carla.py:4-5``
expects."""
