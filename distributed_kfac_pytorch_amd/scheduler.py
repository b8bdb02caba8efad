"""KFACParamScheduler: step-wise schedules for damping and update frequencies.

Parity with kfac/scheduler.py:1-94 of the reference: writes
`damping = base * damping_alpha ** #(milestones <= step)` and both update
frequencies `= int(base * update_freq_alpha ** #(milestones <= step))` into
`kfac.param_groups[0]`.  Typically stepped once per epoch.  The state dict
holds the same keys as the reference's (every attribute except the KFAC
handle and the schedule callables).
"""

__all__ = ['KFACParamScheduler']


class KFACParamScheduler(object):
    def __init__(self, kfac, damping_alpha=1, damping_schedule=None, update_freq_alpha=1,
                 update_freq_schedule=None, start_step=0):
        self.kfac = kfac
        params = kfac.param_groups[0]
        self.damping_base = params['damping']
        self.damping_alpha = damping_alpha
        self.damping_schedule = damping_schedule
        self.damping_factor_func = self._get_factor_func(damping_schedule, damping_alpha)
        self.factor_update_freq_base = params['factor_update_freq']
        self.inv_update_freq_base = params['inv_update_freq']
        self.update_freq_alpha = update_freq_alpha
        self.update_freq_schedule = update_freq_schedule
        self.update_freq_factor_func = self._get_factor_func(update_freq_schedule,
                                                             update_freq_alpha)
        self._step = start_step

    def state_dict(self):
        return {k: v for k, v in self.__dict__.items() if k != 'kfac' and 'func' not in k}

    def load_state_dict(self, state_dict):
        self.__dict__.update(state_dict)
        self.damping_factor_func = self._get_factor_func(self.damping_schedule,
                                                         self.damping_alpha)
        self.update_freq_factor_func = self._get_factor_func(self.update_freq_schedule,
                                                             self.update_freq_alpha)

    @staticmethod
    def _get_factor_func(schedule, alpha):
        milestones = sorted(schedule, reverse=True) if schedule else []
        if schedule is not None:
            schedule.sort(reverse=True)   # reference sorts the caller's list in place

        def factor(step):
            f = 1.0
            for m in milestones:
                if step >= m:
                    f *= alpha
            return f
        return factor

    def step(self, step=None):
        self._step = self._step + 1 if step is None else step
        params = self.kfac.param_groups[0]
        params['damping'] = self.damping_base * self.damping_factor_func(self._step)
        f = self.update_freq_factor_func(self._step)
        params['factor_update_freq'] = int(self.factor_update_freq_base * f)
        params['inv_update_freq'] = int(self.inv_update_freq_base * f)
