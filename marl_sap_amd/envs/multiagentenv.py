"""Env plugin base (reference: envs/multiagentenv.py:1-60).

The reference's abstract interface: the methods a concrete env must provide raise
NotImplementedError, as there.  The per-agent accessors default to indexing the batch
getters (a subclass that implements get_obs / get_avail_actions gets them), and
get_env_info is the reference's dictionary.  The batched HIP envs (assign_env.py,
real_env.py) implement the batch getters over every env of the handle."""


class MultiAgentEnv:
    def step(self, actions):
        """Returns reward, terminated, info."""
        raise NotImplementedError

    def get_obs(self):
        """Returns all agent observations in a list."""
        raise NotImplementedError

    def get_obs_agent(self, agent_id):
        """Returns the observation of agent_id (default: get_obs()[agent_id])."""
        return self.get_obs()[agent_id]

    def get_obs_size(self):
        """Returns the shape of the observation."""
        raise NotImplementedError

    def get_state(self):
        raise NotImplementedError

    def get_state_size(self):
        """Returns the shape of the state."""
        raise NotImplementedError

    def get_avail_actions(self):
        raise NotImplementedError

    def get_avail_agent_actions(self, agent_id):
        """Returns the available actions of agent_id (default: get_avail_actions()[agent_id])."""
        return self.get_avail_actions()[agent_id]

    def get_total_actions(self):
        """Returns the number of actions an agent could ever take (discrete, one dimension)."""
        raise NotImplementedError

    def reset(self):
        """Returns initial observations and states."""
        raise NotImplementedError

    def render(self):
        raise NotImplementedError

    def close(self):
        raise NotImplementedError

    def seed(self):
        raise NotImplementedError

    def save_replay(self):
        raise NotImplementedError

    def get_env_info(self):
        return {"state_shape": self.get_state_size(), "obs_shape": self.get_obs_size(),
                "m": self.get_total_actions(), "n": self.n, "T": self.T}
