"""mujoco_warp_amd: MI355X-native batched MuJoCo stepper.

Public API mirrors `import mujoco_warp as mjw` (mujoco_warp/__init__.py:26-112)
for the `step` path: put_model / put_data / make_data / step / forward / stage
functions / get_data_into / reset_data / override_model, plus the enums and
Model/Data containers.  Compute runs in hand-written HIP kernels (gfx950)
behind the C ABI in include/mjw_amd.h; see DESIGN.md.
"""

from .forward import ctrl_noise
from .forward import euler
from .forward import forward
from .forward import fwd_acceleration
from .forward import fwd_actuation
from .forward import fwd_position
from .forward import fwd_velocity
from .forward import implicit
from .forward import sensor_acc
from .forward import sensor_pos
from .forward import sensor_vel
from .forward import solve
from .forward import step
from .forward import rungekutta4
from .forward import step1
from .forward import step2
from .io import find_keys
from .io import get_data_into
from .io import make_trajectory
from .io import make_data
from .io import override_model
from .io import put_data
from .io import put_model
from .io import reset_data
from .mjcf import MjData
from .mjcf import MjModel
from .mjcf import load_model
from .mjcf import load_model_from_string
from .mjcf import reset_data_keyframe
from .stages import camlight
from .stages import collision
from .stages import CollisionContext
from .stages import create_collision_context
from .stages import nxn_broadphase
from .stages import primitive_narrowphase
from .stages import sap_broadphase
from .stages import com_pos
from .stages import com_vel
from .stages import crb
from .stages import energy_pos
from .stages import energy_vel
from .stages import factor_m
from .stages import flex
from .stages import jac
from .stages import kinematics
from .stages import make_constraint
from .stages import passive
from .stages import rne
from .stages import rne_postconstraint
from .stages import set_const
from .stages import set_const_0
from .stages import set_const_fixed
from .stages import set_length_range
from .stages import deriv_smooth_vel
from .stages import solve_m
from .stages import subtree_vel
from .stages import tendon
from .stages import transmission
from .stages import xfrc_accumulate
from .support import contact_force
from .support import get_state
from .support import efc_J_csr
from .support import mul_m
from .support import set_state
from .support import state_size
from .types import BiasType
from .types import Callback
from .types import BroadphaseFilter
from .types import BroadphaseType
from .types import CamLightType
from .types import ConeType
from .types import ConstraintState
from .types import ConstraintType
from .types import Contact
from .types import Constraint
from .types import Data
from .types import DisableBit
from .types import DynType
from .types import EnableBit
from .types import GainType
from .types import GeomType
from .types import IntegratorType
from .types import JointType
from .types import Model
from .types import Option
from .types import SolverType
from .types import State
from .types import Statistic
from .types import TrnType
