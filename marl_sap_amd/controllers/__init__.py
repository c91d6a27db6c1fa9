from .basic_controller import BasicMAC
from .jumpstart_controller import JumpstartMAC

REGISTRY = {"basic_mac": BasicMAC, "jumpstart_mac": JumpstartMAC}
