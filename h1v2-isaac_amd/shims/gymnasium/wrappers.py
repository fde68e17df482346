class RecordVideo:
    def __init__(self, env, *args, **kwargs):
        raise NotImplementedError("video recording needs a renderer; the MI355X build has none (run without --video)")
