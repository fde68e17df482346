"""biped_tasks: the H1-2 12-DoF velocity tasks registered against the MI355X env."""
