class FrameStack:
    pass
