"""MI355X-native FaithDiff: drop-in for the reference's ``FaithDiff`` package surface
(create_FaithDiff_model.FaithDiff_pipeline, pipelines.pipeline_FaithDiff_tlc, models.*)."""
