"""Task registry mirroring isaacgymenvs/tasks/__init__.py (the tasks on the BASELINE.json hot path)."""
from .allegro_hand import AllegroHand
from .allegro_kuka import AllegroKuka, AllegroKukaRegrasping, AllegroKukaReorientation, AllegroKukaThrow
from .ur5sih_multi_object_manipulation import Ur5SihMultiObjectManipulation

isaacgym_task_map = {
    "Ur5SihMultiObjectManipulation": Ur5SihMultiObjectManipulation,
    "AllegroHand": AllegroHand,
    "AllegroKuka": AllegroKuka,                  # subtask from cfg env.subtask (tasks/__init__.py resolver)
    "AllegroKukaRegrasping": AllegroKukaRegrasping,
    "AllegroKukaReorientation": AllegroKukaReorientation,
    "AllegroKukaThrow": AllegroKukaThrow,
}
