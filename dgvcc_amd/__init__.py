"""dgvcc_amd — MI355X-native (gfx950 HIP) implementation of the DGVCC crowd-density
training hot path, drop-in behind the reference's models.models / models.models2 /
trainers.dgtrainer / losses.bl / utils.dmap_gen interfaces."""
__version__ = "0.1.0"
