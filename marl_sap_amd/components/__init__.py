from .episode_buffer import EpisodeBatch, ReplayBuffer
from .transforms import OneHot
from .epsilon_schedules import DecayThenFlatSchedule
