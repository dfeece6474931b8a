"""Collection and result names a custom rule module needs (the reference's environment/constants.py keys)."""
DEFAULTS = 'Defaults'
WALL = 'Wall'
WALLS = 'Walls'
AGENT = 'Agent'
COLLISION = 'Collisions'
VALID = True
NOT_VALID = False
VALUE_NO_POS = (-9999, -9999)
NOOP = 'Noop'
