"""Import-only stand-in: the reference's data loaders are never called by the fixture script."""
import types

transforms = types.ModuleType("torchvision.transforms")
