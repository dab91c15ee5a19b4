"""shai_amd.supervisor"""
