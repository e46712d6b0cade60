"""Goal-tolerance schedule, restated from envs/goal_tolerance.py:8-56 (host scalar).

The current tolerance is handed to the step/reset kernels as a scalar argument.
"""
import numpy as np


class GoalTolerance(object):
    VALID = ("constant", "linear", "decay")

    def __init__(self, goal_tolerance_parameters):
        p = goal_tolerance_parameters
        self.goal_tolerance_parameters = p
        self.inc_tol_obs = p["inc_tol_obs"]          # stored, never applied (reference Q11)
        self.init_tol = p["initial_tol"]
        self.final_tol = p["final_tol"]
        self.N_ts = p["N_ts"]
        self.function = p["function"]
        assert self.function in self.VALID, "Not a valid function. Choose constant, linear or decay."
        if self.function == "linear":
            self.a = (self.final_tol - self.init_tol) / self.N_ts
            self.b = self.init_tol
        if self.function == "decay":
            self.a = self.init_tol
            self.r = 1 - np.power((self.final_tol / self.init_tol), 1 / self.N_ts)
        self.set_tol_value = p["set_tol"]
        self.current_tol = self.init_tol if self.set_tol_value == 0 else self.set_tol_value
        self.training_step = 0

    def update(self, timestep):
        if self.set_tol_value == 0:
            if self.function == "linear" and timestep <= self.N_ts:
                self.current_tol = self.a * timestep + self.b
            elif self.function == "decay" and timestep <= self.N_ts:
                self.current_tol = self.a * np.power(1 - self.r, timestep)
            else:
                self.current_tol = self.final_tol
        else:
            self.current_tol = self.set_tol_value

    def get_tol(self):
        return self.current_tol
