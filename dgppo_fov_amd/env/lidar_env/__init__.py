from .base import LidarEnv, LidarEnvState
from .lidar_spread import LidarSpread
from .lidar_target import LidarTarget
from .lidar_bicycle_target import LidarBicycleTarget
from .lidar_omni_target import LidarOmniTarget
from .lidar_line import LidarLine
