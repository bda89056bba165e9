"""Task registry mirroring isaacgymenvs/tasks/__init__.py (hand-arm path only)."""
from .ur5sih_multi_object_manipulation import Ur5SihMultiObjectManipulation

isaacgym_task_map = {
    "Ur5SihMultiObjectManipulation": Ur5SihMultiObjectManipulation,
}
